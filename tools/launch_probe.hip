// Diagnostics (r06): what a launch of the batched kernel's shape
// pays outside its workgroups' lives. Back-to-back launches of a fixed-duration kernel
// (256 workgroups x 256 threads, ~80K cycles each: the lean mlp512 kernel's shape) on
// one stream, timed by HIP events; every workgroup stamps its start and end with the
// 100 MHz wall clock, so per launch: span = last end - first start, start spread, end
// spread, and event time - span = what happens between launches. Variants add one
// property of the real kernel at a time: dynamic LDS (the lean kernel asks ~100 KB),
// the action store at the end (16 rows x 12 floats per workgroup), the weight stream
// (each workgroup reads the 2.37 MB weight set once, as the kernel does through L2),
// kernel arguments preloaded into SGPRs.
// Build: hipcc -O3 --offload-arch=gfx950 -mllvm -amdgpu-kernarg-preload-count=16 launch_probe.hip -o launch_probe.bin
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

struct Args {
  unsigned long long *stamps;  // [launch][wg][2]
  const float4 *w;             // weights to stream (nullptr: none)
  float *act;                  // action rows (nullptr: none)
  int nw4;                     // float4s of w
  long long cycles;
  int launch;
};

template <bool LDS, bool STREAM, bool STORE>
__global__ __launch_bounds__(256) void probe_k(Args a) {
  extern __shared__ float4 lds[];
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  const long long c0 = clock64();
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  if (STREAM) {  // the weight set, once per workgroup, 1 KiB per wave instruction
    for (int i = threadIdx.x; i < a.nw4; i += 256) {
      const float4 v = a.w[i];
      acc.x += v.x;
      acc.y += v.y;
    }
  }
  if (LDS) {
    lds[threadIdx.x] = acc;
    __syncthreads();
    acc = lds[(threadIdx.x + 1) & 255];
  }
  while (clock64() - c0 < a.cycles) {
  }
  if (STORE && threadIdx.x < 16 * 12) a.act[blockIdx.x * 16 * 12 + threadIdx.x] = acc.x + acc.y;
  if (threadIdx.x == 0) {
    const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    a.stamps[((size_t)a.launch * gridDim.x + blockIdx.x) * 2] = t0;
    a.stamps[((size_t)a.launch * gridDim.x + blockIdx.x) * 2 + 1] = t1;
  }
  if (acc.z == 12345.f) a.act[0] = acc.w;  // (keeps the loads)
}

template <bool LDS, bool STREAM, bool STORE>
void run(const char *name, size_t lds_bytes, Args a, hipStream_t s, int n) {
  auto k = probe_k<LDS, STREAM, STORE>;
  if (lds_bytes > 64 * 1024) hipFuncSetAttribute((const void *)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_bytes);
  const int G = 256;
  for (int i = 0; i < 50; ++i) {
    a.launch = 0;
    hipLaunchKernelGGL(k, dim3(G), dim3(256), lds_bytes, s, a);
  }
  hipStreamSynchronize(s);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0, s);
  for (int i = 0; i < n; ++i) {
    a.launch = i;
    hipLaunchKernelGGL(k, dim3(G), dim3(256), lds_bytes, s, a);
  }
  hipEventRecord(e1, s);
  hipEventSynchronize(e1);
  float ms = 0.f;
  hipEventElapsedTime(&ms, e0, e1);
  std::vector<unsigned long long> st((size_t)n * G * 2);
  hipMemcpy(st.data(), a.stamps, st.size() * 8, hipMemcpyDeviceToHost);
  std::vector<double> span, ss, es, life;
  for (int i = 0; i < n; ++i) {
    unsigned long long s0 = ~0ull, s1 = 0, e0_ = ~0ull, e1_ = 0;
    std::vector<double> lf;
    for (int g = 0; g < G; ++g) {
      const unsigned long long t0 = st[((size_t)i * G + g) * 2], t1 = st[((size_t)i * G + g) * 2 + 1];
      s0 = std::min(s0, t0);
      s1 = std::max(s1, t0);
      e0_ = std::min(e0_, t1);
      e1_ = std::max(e1_, t1);
      lf.push_back((t1 - t0) * 0.01);
    }
    std::sort(lf.begin(), lf.end());
    span.push_back((e1_ - s0) * 0.01);
    ss.push_back((s1 - s0) * 0.01);
    es.push_back((e1_ - e0_) * 0.01);
    life.push_back(lf[G / 2]);
  }
  auto med = [](std::vector<double> v) {
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
  };
  const double ev = ms * 1000.0 / n;
  std::printf("%-34s event %.2f us  span %.2f  wg life %.2f  start spread %.2f  end spread %.2f  event-span %.2f\n",
              name, ev, med(span), med(life), med(ss), med(es), ev - med(span));
}

int main() {
  hipStream_t s;
  hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  const int n = 1000, G = 256;
  Args a{};
  hipMalloc(&a.stamps, (size_t)n * G * 2 * 8);
  const int nw4 = 2370000 / 16;
  float4 *w;
  hipMalloc(&w, (size_t)nw4 * 16);
  hipMemset(w, 0, (size_t)nw4 * 16);
  hipMalloc(&a.act, (size_t)G * 16 * 12 * 4);
  a.nw4 = nw4;
  a.cycles = 80000;
  a.w = w;
  run<false, false, false>("spin", 0, a, s, n);
  run<true, false, false>("spin + 64 KB LDS", 64 * 1024, a, s, n);
  run<true, false, false>("spin + 100 KB LDS", 100 * 1024, a, s, n);
  run<true, false, false>("spin + 160 KB LDS", 160 * 1024, a, s, n);
  run<false, false, true>("spin + action store", 0, a, s, n);
  run<false, true, false>("spin + weight stream", 0, a, s, n);
  run<true, true, true>("spin + 100 KB LDS + stream + store", 100 * 1024, a, s, n);
  a.cycles = 76000;
  run<true, true, true>("(76K cycles) all three", 100 * 1024, a, s, n);
  return 0;
}
