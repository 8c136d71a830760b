// Diagnostics: host -> GPU -> host round-trip floor of a live (resident) kernel,
// by where the request word lives. One workgroup, wave 0 lane 0 polls the
// request word, then writes the done word (vector stores, system scope) into
// pinned host memory; the host spins on it. Every spin on either side is bounded.
//   host   request in pinned host memory (what the resident kernel does today)
//   fgvram request in fine-grained device memory the host writes through its mapping
// Build: hipcc -O3 --offload-arch=gfx950 pcie_echo.hip -o pcie_echo
#include <hip/hip_runtime.h>
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

#define CK(x)                                                          \
  do {                                                                 \
    hipError_t e_ = (x);                                               \
    if (e_ != hipSuccess) {                                            \
      std::printf("%s: %s\n", #x, hipGetErrorString(e_));              \
      return 1;                                                        \
    }                                                                  \
  } while (0)

// polls req until it equals epoch e, answers done = e, for e = 1..n; leaves on a
// poll that outlives ~2 s (100 MHz s_memrealtime) so the grid always drains
__global__ void echo_k(const unsigned *req, unsigned *done, int n) {
  if (threadIdx.x != 0) return;
  for (int e = 1; e <= n; ++e) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    for (;;) {
      const unsigned v = __hip_atomic_load(req, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      if (v == (unsigned)e) break;
      if (__builtin_amdgcn_s_memrealtime() - t0 > 200000000ull) return;
    }
    __hip_atomic_store(done, (unsigned)e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

static int run(const char *name, unsigned *h_req, const unsigned *d_req, volatile unsigned *h_done,
               unsigned *d_done, int n) {
  *reinterpret_cast<volatile unsigned *>(h_req) = 0;
  *h_done = 0;
  hipLaunchKernelGGL(echo_k, dim3(1), dim3(64), 0, 0, d_req, d_done, n);
  std::vector<double> ts;
  ts.reserve(n);
  for (int e = 1; e <= n; ++e) {
    const auto t0 = std::chrono::steady_clock::now();
    __atomic_store_n(h_req, (unsigned)e, __ATOMIC_RELEASE);
    bool ok = false;
    for (long it = 0; it < 400000000L; ++it)
      if (*h_done == (unsigned)e) {
        ok = true;
        break;
      }
    const auto t1 = std::chrono::steady_clock::now();
    if (!ok) {
      std::printf("%s: no answer for epoch %d\n", name, e);
      break;
    }
    ts.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
  }
  CK(hipDeviceSynchronize());
  if (ts.size() < 100) return 1;
  std::vector<double> s(ts.begin() + 100, ts.end());
  std::sort(s.begin(), s.end());
  std::printf("%-8s round trip p50 %.2f us  p99 %.2f us  min %.2f us  (%zu)\n", name, s[s.size() / 2],
              s[s.size() * 99 / 100], s[0], s.size());
  return 0;
}

int main() {
  const int n = 5000;
  unsigned *h_done, *d_done, *h_req, *d_req;
  CK(hipHostMalloc((void **)&h_done, 4096, hipHostMallocMapped));
  CK(hipHostGetDevicePointer((void **)&d_done, h_done, 0));
  CK(hipHostMalloc((void **)&h_req, 4096, hipHostMallocMapped));
  CK(hipHostGetDevicePointer((void **)&d_req, h_req, 0));
  if (run("host", h_req, d_req, h_done, d_done, n)) return 1;

  unsigned *v_req = nullptr;
  if (hipExtMallocWithFlags((void **)&v_req, 4096, hipDeviceMallocFinegrained) != hipSuccess) {
    std::printf("fgvram: hipExtMallocWithFlags failed\n");
    return 0;
  }
  hipPointerAttribute_t at{};
  CK(hipPointerGetAttributes(&at, v_req));
  std::printf("fgvram: type %d device %p host %p\n", (int)at.type, at.devicePointer, at.hostPointer);
  if (!at.hostPointer) {
    std::printf("fgvram: no host mapping\n");
    return 0;
  }
  return run("fgvram", static_cast<unsigned *>(at.hostPointer), v_req, h_done, d_done, n);
}
