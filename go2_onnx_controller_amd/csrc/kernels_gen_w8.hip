// Generic batched body, 8 waves per workgroup (see kernels_gen.inc).
#define GO2PI_GEN_NW 8
#include "kernels_gen.inc"
