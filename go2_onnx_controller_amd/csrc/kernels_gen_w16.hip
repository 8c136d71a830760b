// Generic batched body, 16 waves per workgroup (see kernels_gen.inc).
#define GO2PI_GEN_NW 16
#include "kernels_gen.inc"
