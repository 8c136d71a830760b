// Microbenchmark (diagnostics): cycles per v_mfma_f32_16x16x4_f32 for one wave per
// SIMD (4 waves per workgroup, one workgroup per CU) in the operand forms the
// batched kernel's inner loop uses. Build: hipcc -O3 --offload-arch=gfx950
// tools/mfma_rate.hip -o /tmp/mfma_rate. Prints cycles per MFMA (s_memtime) for:
//   vv   : A and B from VGPRs, 8 independent accumulators
//   av   : A from AGPRs (inline asm operand "a"), B from VGPR
//   vv+l : vv with 1 ds_read_b128 per 32 MFMAs feeding the B operands
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int MODE>
__global__ __launch_bounds__(256) void rate(float *out, unsigned long long *cyc, int iters) {
  __shared__ float lds[1024];
  const int lane = threadIdx.x & 63;
  lds[threadIdx.x] = (float)lane;
  __syncthreads();
  f32x4 acc[8];
  for (int i = 0; i < 8; ++i) acc[i] = f32x4{0, 0, 0, 0};
  float a[8], b[4];
  for (int i = 0; i < 8; ++i) a[i] = 1e-3f * (lane + i);
  for (int j = 0; j < 4; ++j) b[j] = 1e-3f * (lane - j);
  const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < iters; ++it) {
    if constexpr (MODE == 2) {  // one LDS read per 32 MFMAs, consumed by the next iteration's MFMAs
      const float4 v = *reinterpret_cast<const float4 *>(lds + ((lane + it) & 255) * 4);
      b[0] = v.x;
      b[1] = v.y;
      b[2] = v.z;
      b[3] = v.w;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        if constexpr (MODE == 1) {
          asm volatile("v_mfma_f32_16x16x4_f32 %0, %1, %2, %0" : "+a"(acc[i]) : "a"(a[i]), "v"(b[j]));
        } else {
          acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i], b[j], acc[i], 0, 0, 0);
        }
      }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  float s = 0;
  for (int i = 0; i < 8; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[blockIdx.x * 256 + threadIdx.x] = s;
  if (threadIdx.x == 0) {
    cyc[2 * blockIdx.x] = t1 - t0;
    cyc[2 * blockIdx.x + 1] = r1 - r0;  // 100 MHz ticks
  }
}

int main() {
  const int blocks = 256, iters = 65536;  // ~30 ms per launch: long enough for the clock to settle
  printf("start\n");
  fflush(stdout);
  float *out;
  unsigned long long *cyc;
  hipMalloc(&out, sizeof(float) * blocks * 256);
  hipMalloc(&cyc, sizeof(unsigned long long) * blocks * 2);
  unsigned long long h[512];
  const char *names[3] = {"vv", "av", "vv+l"};
  for (int mode = 0; mode < 3; ++mode) {
    for (int rep = 0; rep < 5; ++rep) {
      if (mode == 0) hipLaunchKernelGGL(rate<0>, dim3(blocks), dim3(256), 0, 0, out, cyc, iters);
      if (mode == 1) hipLaunchKernelGGL(rate<1>, dim3(blocks), dim3(256), 0, 0, out, cyc, iters);
      if (mode == 2) hipLaunchKernelGGL(rate<2>, dim3(blocks), dim3(256), 0, 0, out, cyc, iters);
    }
    const hipError_t e = hipDeviceSynchronize();
    if (e != hipSuccess) {
      printf("mode %s: %s\n", names[mode], hipGetErrorString(e));
      return 1;
    }
    hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
    unsigned long long s = 0, r = 0;
    for (int i = 0; i < blocks; ++i) {
      s += h[2 * i];
      r += h[2 * i + 1];
    }
    printf("%-5s cycles per MFMA (mean over workgroups): %.2f  clock %.3f GHz  ns per MFMA %.2f\n", names[mode],
           (double)s / blocks / (iters * 32.0), (double)s / r * 0.1, (double)r * 10.0 / blocks / (iters * 32.0));
    fflush(stdout);
  }
  return 0;
}
