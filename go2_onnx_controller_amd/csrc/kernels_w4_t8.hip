// 4-wave pipeline instantiations, 8 tiles per wave (see kernels_w4.inc).
#define GO2PI_W4_TPW 8
#include "kernels_w4.inc"
