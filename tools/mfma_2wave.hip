// Microbenchmark (diagnostics): with TWO waves per SIMD, does one wave's VALU work
// (an Elu epilogue's instruction mix) run beside the other wave's
// v_mfma_f32_16x16x4_f32 stream without slowing it? (tools/mfma_valu.hip measured the
// one-wave case: every VALU instruction in an MFMA gap adds 4-13 cycles.) 256
// workgroups of 8 waves, waves w and w + 4 on one SIMD.
//   mode 0: waves 0-3 MFMA only, waves 4-7 idle (exit at once)  -> the pipe alone
//   mode 1: waves 0-3 MFMA, waves 4-7 an epilogue mix (accvgpr read, pk_mul, exp,
//           pk_add, cmp + cndmask per element pair) for their whole life
//   mode 2: all 8 waves MFMA (how the pipe is split between two waves)
//   mode 3: waves 4-7 the epilogue mix alone (waves 0-3 exit at once)
// Prints, per wave group, cycles per MFMA (s_memtime) and, for the VALU waves, cycles
// per epilogue element.
// Build: hipcc -O3 --offload-arch=gfx950 tools/mfma_2wave.hip -o tools/mfma_2wave.bin
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ void mfma_block(f32x4 (&acc)[8], const float (&a)[8], const float (&b)[4]) {
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int i = 0; i < 8; ++i)
      asm volatile("v_mfma_f32_16x16x4_f32 %0, %1, %2, %0" : "+a"(acc[i]) : "v"(a[i]), "v"(b[j]));
}

// 8 elements of an Elu epilogue (4 packed pairs), registers of its own
__device__ __forceinline__ void epi_block(f32x4 &src, f32x2 (&x)[4], float (&o)[8]) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    asm volatile("v_accvgpr_read_b32 %0, %2\n\tv_accvgpr_read_b32 %1, %3"
                 : "=v"(x[q].x), "=v"(x[q].y) : "a"(src[q & 3]), "a"(src[(q + 1) & 3]));
    f32x2 t = x[q] * f32x2{1.4426950408889634f, 1.4426950408889634f};
    float e0, e1;
    asm volatile("v_exp_f32 %0, %2\n\tv_exp_f32 %1, %3" : "=v"(e0), "=v"(e1) : "v"(t.x), "v"(t.y));
    f32x2 e = f32x2{e0, e1} - 1.f;
    asm volatile("v_cmp_lt_f32 vcc, 0, %2\n\tv_cndmask_b32 %0, %3, %2, vcc\n\t"
                 "v_cmp_lt_f32 vcc, 0, %4\n\tv_cndmask_b32 %1, %5, %4, vcc"
                 : "=v"(o[2 * q]), "=v"(o[2 * q + 1]) : "v"(x[q].x), "v"(e.x), "v"(x[q].y), "v"(e.y) : "vcc");
  }
}

template <int MODE>
__global__ __launch_bounds__(512) void k2(float *out, unsigned long long *cyc, int iters) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const bool mf = (wave < 4 || MODE == 2) && MODE != 3;
  if ((MODE == 0 && !mf) || (MODE == 3 && wave < 4)) return;
  float s = 0.f;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  if (mf) {
    f32x4 acc[8];
    for (int i = 0; i < 8; ++i) acc[i] = f32x4{0, 0, 0, 0};
    float a[8], b[4];
    for (int i = 0; i < 8; ++i) a[i] = 1e-3f * (lane + i);
    for (int j = 0; j < 4; ++j) b[j] = 1e-3f * (lane - j);
    for (int it = 0; it < iters; ++it) mfma_block(acc, a, b);
    for (int i = 0; i < 8; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  } else {
    f32x4 src = {1.f * lane, -2.f, 3.f, -4.f};
    asm volatile("" : "+a"(src));
    f32x2 x[4];
    float o[8] = {};
    // 32 elements per 32-MFMA block of the partner (far denser than the lean kernel's
    // 32 per 1024), so that the VALU wave stays busy for about the partner's whole life
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        epi_block(src, x, o);
        asm volatile("" : "+v"(o[0]), "+v"(o[3]), "+v"(o[7]));
      }
    }
    for (int q = 0; q < 8; ++q) s += o[q];
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * 512 + threadIdx.x] = s;
  if (lane == 0) cyc[blockIdx.x * 8 + wave] = t1 - t0;
}

template <int MODE>
static void run(const char *name, float *out, unsigned long long *cyc) {
  const int blocks = 256, iters = 4096;
  unsigned long long h[256 * 8];
  hipMemset(cyc, 0, sizeof(h));
  for (int rep = 0; rep < 3; ++rep) hipLaunchKernelGGL((k2<MODE>), dim3(blocks), dim3(512), 0, 0, out, cyc, iters);
  if (hipDeviceSynchronize() != hipSuccess) {
    printf("%s failed\n", name);
    return;
  }
  hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
  double lo = 0, hi = 0;
  for (int i = 0; i < blocks; ++i)
    for (int w = 0; w < 8; ++w) (w < 4 ? lo : hi) += (double)h[i * 8 + w];
  lo /= blocks * 4.0;
  hi /= blocks * 4.0;
  printf("%-28s waves0-3: %.2f cyc/MFMA", name, lo / (iters * 32.0));
  if (MODE == 1 || MODE == 3) printf("  waves4-7: %.2f cyc/element (%.0f cycles)", hi / (iters * 32.0), hi);
  if (MODE == 2) printf("  waves4-7: %.2f cyc/MFMA", hi / (iters * 32.0));
  printf("\n");
  fflush(stdout);
}

int main() {
  float *out;
  unsigned long long *cyc;
  hipMalloc(&out, sizeof(float) * 256 * 512);
  hipMalloc(&cyc, sizeof(unsigned long long) * 256 * 8);
  run<0>("mfma alone", out, cyc);
  run<1>("mfma + partner epilogue", out, cyc);
  run<2>("mfma + partner mfma", out, cyc);
  run<3>("epilogue alone", out, cyc);
  return 0;
}
