// Diagnostics: per-launch floor of back-to-back kernels on one stream (HIP events),
// by grid shape, dynamic LDS and kernarg size — what a one-launch-per-step design
// pays between steps on this stack. Build: hipcc -O3 --offload-arch=gfx950 launch_gap.hip
#include <hip/hip_runtime.h>
#include <cstdio>

struct Big { char b[800]; };

__global__ void empty_k(int *p) { if (p && threadIdx.x == 9999) p[0] = 1; }
__global__ void big_arg_k(Big a, int *p) { if (p && threadIdx.x == 9999) p[0] = a.b[blockIdx.x & 511]; }
__global__ void lds_k(int *p) {
  extern __shared__ int s[];
  if (threadIdx.x == 0) s[0] = blockIdx.x;
  __syncthreads();
  if (p && threadIdx.x == 9999) p[0] = s[0];
}
__global__ void spin_k(int *p, long long cycles) {  // ~fixed-duration kernel
  long long t0 = clock64();
  while (clock64() - t0 < cycles) {}
  if (p && threadIdx.x == 9999) p[0] = 1;
}

template <class F>
static float timeit(hipStream_t s, int n, F f) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int i = 0; i < 50; ++i) f();
  hipStreamSynchronize(s);
  hipEventRecord(a, s);
  for (int i = 0; i < n; ++i) f();
  hipEventRecord(b, s);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  return ms * 1000.f / n;
}

int main() {
  hipStream_t s;
  hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  const int n = 2000;
  Big big{};
  hipFuncSetAttribute((const void *)lds_k, hipFuncAttributeMaxDynamicSharedMemorySize, 80 * 1024);
  printf("empty 1x64        %.2f us\n", timeit(s, n, [&] { hipLaunchKernelGGL(empty_k, dim3(1), dim3(64), 0, s, nullptr); }));
  printf("empty 256x512     %.2f us\n", timeit(s, n, [&] { hipLaunchKernelGGL(empty_k, dim3(256), dim3(512), 0, s, nullptr); }));
  printf("bigarg 256x512    %.2f us\n", timeit(s, n, [&] { hipLaunchKernelGGL(big_arg_k, dim3(256), dim3(512), 0, s, big, nullptr); }));
  printf("lds74K 256x512    %.2f us\n", timeit(s, n, [&] { hipLaunchKernelGGL(lds_k, dim3(256), dim3(512), 74 * 1024, s, nullptr); }));
  for (long long cyc : {20000LL, 100000LL}) {
    printf("spin %lld cyc 256x512  %.2f us\n", cyc,
           timeit(s, 500, [&] { hipLaunchKernelGGL(spin_k, dim3(256), dim3(512), 0, s, nullptr, cyc); }));
    printf("spin %lld cyc 1x64     %.2f us\n", cyc,
           timeit(s, 500, [&] { hipLaunchKernelGGL(spin_k, dim3(1), dim3(64), 0, s, nullptr, cyc); }));
  }
  // the lean kernel's shape (256 workgroups of 256 threads, ~80K cycles each), on one
  // stream, then the same launches captured once in a hipGraph and replayed
  const long long cyc = 80000;
  const float plain = timeit(s, 500, [&] { hipLaunchKernelGGL(spin_k, dim3(256), dim3(256), 0, s, nullptr, cyc); });
  printf("spin %lld cyc 256x256  %.2f us\n", cyc, plain);
  hipGraph_t g;
  hipGraphExec_t ge;
  hipStreamBeginCapture(s, hipStreamCaptureModeGlobal);
  for (int i = 0; i < 100; ++i) hipLaunchKernelGGL(spin_k, dim3(256), dim3(256), 0, s, nullptr, cyc);
  hipStreamEndCapture(s, &g);
  hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
  printf("spin %lld cyc 256x256 graph x100  %.2f us\n", cyc, timeit(s, 5, [&] { hipGraphLaunch(ge, s); }) / 100.f);
  return 0;
}
