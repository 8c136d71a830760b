// 4-wave pipeline instantiations, 4 tiles per wave (see kernels_w4.inc).
#define GO2PI_W4_TPW 4
#include "kernels_w4.inc"
