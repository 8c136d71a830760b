// Microbenchmark (diagnostics): does VALU work between v_mfma_f32_16x16x4_f32
// instructions of one wave per SIMD hide behind the MFMA pipe? (The batched
// kernel's epilogue is VALU work that the own phase could carry.) One workgroup of
// 4 waves per CU, 256 workgroups; each wave issues 32 MFMAs per iteration onto 8
// AGPR accumulators (A, B from VGPRs, as in the kernel) and, after every MFMA, NV
// independent filler instructions of kind KIND on registers of their own:
//   0 v_add_f32, 1 v_exp_f32, 2 v_pk_add_f32, 3 v_accvgpr_read_b32 (of an AGPR
//   that no MFMA writes), 4 v_cndmask_b32 after v_cmp (the Elu select pair)
// Prints cycles per MFMA (s_memtime); 32.0 = the MFMA pipe's issue rate.
// Build: hipcc -O3 --offload-arch=gfx950 tools/mfma_valu.hip -o /tmp/mfma_valu
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

template <int NV, int KIND>
__device__ __forceinline__ void filler(float (&r)[8], f32x2 (&p)[4], f32x4 &spare, int m) {
#pragma unroll
  for (int q = 0; q < NV; ++q) {
    const int k = (m * NV + q) & 7;
    if constexpr (KIND == 0) asm volatile("v_add_f32 %0, 1.0, %0" : "+v"(r[k]));
    if constexpr (KIND == 1) asm volatile("v_exp_f32 %0, %0" : "+v"(r[k]));
    if constexpr (KIND == 2) asm volatile("v_pk_add_f32 %0, %0, 1.0 op_sel_hi:[1,0]" : "+v"(p[k & 3]));
    if constexpr (KIND == 3) asm volatile("v_accvgpr_read_b32 %0, %1" : "=v"(r[k]) : "a"(spare[k & 3]));
    if constexpr (KIND == 4)
      asm volatile("v_cmp_lt_f32 vcc, 0, %0\n\tv_cndmask_b32 %0, %1, %0, vcc" : "+v"(r[k]) : "v"(r[(k + 1) & 7]) : "vcc");
  }
}

template <int NV, int KIND>
__global__ __launch_bounds__(256) void rate(float *out, unsigned long long *cyc, int iters) {
  const int lane = threadIdx.x & 63;
  f32x4 acc[8];
  for (int i = 0; i < 8; ++i) acc[i] = f32x4{0, 0, 0, 0};
  float a[8], b[4], r[8];
  f32x2 p[4];
  f32x4 spare = {1.f * lane, 2.f, 3.f, 4.f};
  for (int i = 0; i < 8; ++i) a[i] = 1e-3f * (lane + i), r[i] = -1e-3f * (lane + i);
  for (int j = 0; j < 4; ++j) b[j] = 1e-3f * (lane - j), p[j] = f32x2{0.5f * j, 0.25f * lane};
  asm volatile("" : "+a"(spare));
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        asm volatile("v_mfma_f32_16x16x4_f32 %0, %1, %2, %0" : "+a"(acc[i]) : "v"(a[i]), "v"(b[j]));
        filler<NV, KIND>(r, p, spare, j * 8 + i);
      }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0;
  for (int i = 0; i < 8; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3] + r[i];
  for (int j = 0; j < 4; ++j) s += p[j].x + p[j].y;
  out[blockIdx.x * 256 + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int NV, int KIND>
static void run(const char *name, float *out, unsigned long long *cyc) {
  const int blocks = 256, iters = 16384;
  unsigned long long h[256];
  for (int rep = 0; rep < 3; ++rep) hipLaunchKernelGGL((rate<NV, KIND>), dim3(blocks), dim3(256), 0, 0, out, cyc, iters);
  if (hipDeviceSynchronize() != hipSuccess) {
    printf("%s failed\n", name);
    return;
  }
  hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
  unsigned long long s = 0;
  for (int i = 0; i < blocks; ++i) s += h[i];
  printf("%-14s NV=%d  cycles per MFMA %.2f\n", name, NV, (double)s / blocks / (iters * 32.0));
  fflush(stdout);
}

int main() {
  float *out;
  unsigned long long *cyc;
  hipMalloc(&out, sizeof(float) * 256 * 256);
  hipMalloc(&cyc, sizeof(unsigned long long) * 256);
  run<0, 0>("none", out, cyc);
  run<1, 0>("v_add", out, cyc);
  run<2, 0>("v_add", out, cyc);
  run<4, 0>("v_add", out, cyc);
  run<1, 1>("v_exp", out, cyc);
  run<2, 1>("v_exp", out, cyc);
  run<1, 2>("v_pk_add", out, cyc);
  run<2, 2>("v_pk_add", out, cyc);
  run<1, 3>("v_accvgpr_read", out, cyc);
  run<2, 3>("v_accvgpr_read", out, cyc);
  run<1, 4>("cmp+cndmask", out, cyc);
  return 0;
}
