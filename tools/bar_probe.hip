// Diagnostics: can the host write a request straight into device memory (a large-BAR
// mapping of VRAM), and what is the live-kernel round trip then?
//
//   host   request word in pinned host memory, polled by the GPU over PCIe (r04 form:
//          each poll is a PCIe read round trip)
//   vram   request word in fine-grained device memory the host writes through the
//          BAR (a posted PCIe write), polled by the GPU in its own memory
//
// Whether a device allocation is mapped into the host's address space is checked with
// msync() on its page (ENOMEM: not mapped), never by dereferencing it. One workgroup,
// lane 0 polls and answers into pinned host memory; every spin on either side is bounded.
// Build: hipcc -O3 --offload-arch=gfx950 bar_probe.hip -o bar_probe -lhsa-runtime64
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <sys/mman.h>

#include <algorithm>
#include <cerrno>
#include <chrono>
#include <cstdint>
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

static bool mapped(const void *p) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(p) & ~uintptr_t(4095);
  return msync(reinterpret_cast<void *>(a), 4096, MS_ASYNC) == 0;
}

static int run(const char *name, volatile unsigned *h_req, const unsigned *d_req, volatile unsigned *h_done,
               unsigned *d_done, int n) {
  *h_req = 0;
  __atomic_thread_fence(__ATOMIC_SEQ_CST);
  *h_done = 0;
  hipLaunchKernelGGL(echo_k, dim3(1), dim3(64), 0, 0, d_req, d_done, n);
  std::vector<double> ts;
  ts.reserve(n);
  for (int e = 1; e <= n; ++e) {
    const auto t0 = std::chrono::steady_clock::now();
    *h_req = (unsigned)e;
    __atomic_thread_fence(__ATOMIC_SEQ_CST);  // (an sfence: the write-combined BAR store goes out now)
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
  if (ts.size() < 200) return 1;
  std::vector<double> s(ts.begin() + 100, ts.end());
  std::sort(s.begin(), s.end());
  std::printf("%-8s round trip p50 %.2f us  p99 %.2f us  min %.2f us  (%zu)\n", name, s[s.size() / 2],
              s[s.size() * 99 / 100], s[0], s.size());
  return 0;
}

static hsa_status_t find_cpu(hsa_agent_t a, void *data) {
  hsa_device_type_t t;
  if (hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) == HSA_STATUS_SUCCESS && t == HSA_DEVICE_TYPE_CPU) {
    *static_cast<hsa_agent_t *>(data) = a;
    return HSA_STATUS_INFO_BREAK;
  }
  return HSA_STATUS_SUCCESS;
}

int main() {
  const int n = 5000;
  unsigned *h_done, *d_done, *h_req, *d_req;
  CK(hipHostMalloc((void **)&h_done, 4096, hipHostMallocMapped));
  CK(hipHostGetDevicePointer((void **)&d_done, h_done, 0));
  CK(hipHostMalloc((void **)&h_req, 4096, hipHostMallocMapped));
  CK(hipHostGetDevicePointer((void **)&d_req, h_req, 0));
  if (run("host", h_req, d_req, h_done, d_done, n)) return 1;

  int large_bar = -1;
  (void)hipDeviceGetAttribute(&large_bar, hipDeviceAttributeIsLargeBar, 0);
  std::printf("hipDeviceAttributeIsLargeBar: %d\n", large_bar);

  unsigned *v_fg = nullptr, *v_cg = nullptr;
  CK(hipExtMallocWithFlags((void **)&v_fg, 4096, hipDeviceMallocFinegrained));
  CK(hipMalloc((void **)&v_cg, 4096));
  std::printf("fine-grained vram %p host-mapped: %d; coarse vram %p host-mapped: %d\n", (void *)v_fg, (int)mapped(v_fg),
              (void *)v_cg, (int)mapped(v_cg));
  hsa_agent_t cpu{};
  if (hsa_iterate_agents(find_cpu, &cpu) == HSA_STATUS_INFO_BREAK) {
    const hsa_status_t s = hsa_amd_agents_allow_access(1, &cpu, nullptr, v_fg);
    std::printf("hsa_amd_agents_allow_access(cpu, fine-grained vram): %d; host-mapped now: %d\n", (int)s,
                (int)mapped(v_fg));
  }
  if (mapped(v_fg)) {
    CK(hipMemset(v_fg, 0, 4096));
    CK(hipDeviceSynchronize());
    if (run("vram-fg", v_fg, v_fg, h_done, d_done, n)) return 1;
  }
  if (mapped(v_cg)) {
    CK(hipMemset(v_cg, 0, 4096));
    CK(hipDeviceSynchronize());
    if (run("vram-cg", v_cg, v_cg, h_done, d_done, n)) return 1;
  }
  return 0;
}
