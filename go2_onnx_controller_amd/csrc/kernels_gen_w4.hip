// Generic batched body, 4 waves per workgroup (see kernels_gen.inc).
#define GO2PI_GEN_NW 4
#include "kernels_gen.inc"
