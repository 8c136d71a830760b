// 4-wave pipeline instantiations, 2 tiles per wave (see kernels_w4.inc).
#define GO2PI_W4_TPW 2
#include "kernels_w4.inc"
