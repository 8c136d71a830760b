// go2pi engine: C-ABI implementation (include/go2pi.h).
//
// Replaces the onnxruntime session behind ONNXActor
// (onnx_inference/src/cpp/onnx_actor.cpp:6-48) with an MI355X-native runtime:
//  - load: parse the .onnx with our own reader (onnx_model.cpp), lower it to a
//    program of dense layers (+ optional GRU), pack weights once into MFMA
//    fragment order (program.hpp) and upload them to HBM (one arena);
//  - host path (go2pi_run): small batches replay a captured hipGraph whose
//    kernels read the observation from / write the action to pinned,
//    host-mapped staging (no memcpy nodes); larger batches stage through
//    device buffers and launch the fused batched kernel;
//  - device path (go2pi_run_device): enqueue on the caller's stream, no sync.
// No CPU fallback exists: without a HIP device, go2pi_create fails loudly.
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <limits>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <tuple>
#include <vector>

#include <immintrin.h>
#include <sys/mman.h>

#include "../../include/go2pi.h"
#include "onnx_model.hpp"
#include "program.hpp"

static bool gru_lean_on();
namespace {

thread_local std::string g_last_error;

struct HipError : std::runtime_error {
  int code;
  HipError(const std::string &m, int c) : std::runtime_error(m), code(c) {}
};

void hip_check(hipError_t e, const char *what) {
  if (e != hipSuccess) throw HipError(std::string("HIP error in ") + what + ": " + hipGetErrorString(e), GO2PI_E_DEVICE);
}
void hip_check(int e, const char *what) { hip_check(static_cast<hipError_t>(e), what); }

struct ApiError : std::runtime_error {
  int code;
  ApiError(const std::string &m, int c) : std::runtime_error(m), code(c) {}
};

inline int ceil16(int x) { return (x + 15) & ~15; }
inline int ceil64(int x) { return (x + 63) & ~63; }

// Pinned host-mapped blocks are never returned to HIP while the process runs:
// hipHostFree (like hipFree) performs an implicit hipDeviceSynchronize, which
// waits for every live resident kernel of every other engine on the device (and
// never returns while another thread keeps one of them busy). A destroyed
// engine's blocks go to this process-wide cache and the next engine reuses them.
std::mutex g_pin_mu;
std::vector<std::pair<size_t, void *>> g_pin_free;  // (bytes, block)

// bytes: in, the size wanted; out, the size of the block handed out (a reused block
// may be larger), which is what pin_give must get back
void *pin_take(size_t &bytes) {
  bytes = (bytes + 4095) & ~(size_t)4095;
  {
    std::lock_guard<std::mutex> lk(g_pin_mu);
    size_t best = g_pin_free.size();
    for (size_t i = 0; i < g_pin_free.size(); ++i)
      if (g_pin_free[i].first >= bytes && (best == g_pin_free.size() || g_pin_free[i].first < g_pin_free[best].first))
        best = i;
    if (best < g_pin_free.size()) {
      void *p = g_pin_free[best].second;
      bytes = g_pin_free[best].first;
      g_pin_free.erase(g_pin_free.begin() + (long)best);
      return p;
    }
  }
  void *p = nullptr;
  hip_check(hipHostMalloc(&p, bytes, hipHostMallocMapped | hipHostMallocCoherent), "hipHostMalloc");
  return p;
}

void pin_give(void *p, size_t bytes) {
  std::lock_guard<std::mutex> lk(g_pin_mu);
  g_pin_free.emplace_back(bytes, p);
}

// The resident kernels' request ring in fine-grained device memory that the host
// writes through its large-BAR mapping of VRAM: a request then reaches the polling
// wave as posted PCIe writes into the GPU's own memory, instead of the wave reading
// pinned host memory across PCIe (a read round trip per poll). tools/bar_probe.hip,
// profiles/r05_bar_probe.txt: live-kernel host -> GPU -> host round trip p50 1.78 us
// against 2.47 us. Whether an allocation is mapped into the host's address space is
// checked with msync() on its pages, never by touching it; without large BAR the ring
// stays in pinned host memory (GO2PI_REQ_HOST=1 forces that, for A/B). Like pinned
// blocks, these are never freed (hipFree synchronises the device): cached per device.
std::vector<std::tuple<int, size_t, void *>> g_bar_free;  // (device, bytes, block), under g_pin_mu
std::vector<int> g_bar_absent;                            // devices whose VRAM the host cannot map

// true when [p, p + bytes) lies inside mappings of this process that are readable
// and writable from the CPU. ROCm's thunk reserves the GPU's virtual aperture with
// PROT_NONE mappings, so an address range being mapped (msync succeeds) does not make
// it host-accessible: without large BAR a fine-grained VRAM block sits in such a range
// and a host store to it faults. /proc/self/maps gives the protection.
bool host_mapped(const void *p, size_t bytes) {
  uintptr_t a = reinterpret_cast<uintptr_t>(p);
  const uintptr_t end = a + bytes;
  FILE *f = std::fopen("/proc/self/maps", "r");
  if (!f) return false;
  char line[512];
  bool ok = false;
  while (a < end && std::fgets(line, sizeof line, f)) {  // (ascending address order)
    unsigned long lo = 0, hi = 0;
    char perm[8] = {0};
    if (std::sscanf(line, "%lx-%lx %7s", &lo, &hi, perm) != 3) continue;
    if (hi <= a) continue;
    if (lo > a || perm[0] != 'r' || perm[1] != 'w') break;  // a hole, or not read-write
    a = hi;  // covered up to hi; the rest must follow in the next mapping(s)
  }
  ok = a >= end;
  std::fclose(f);
  return ok;
}

// a host-writable device block of at least `bytes` (out: its size) on the current
// device `device`, zeroed; nullptr when the host cannot map this device's memory
void *bar_take(int device, size_t &bytes) {
  bytes = (bytes + 4095) & ~(size_t)4095;
  if (std::getenv("GO2PI_REQ_HOST")) return nullptr;
  void *p = nullptr;
  {
    std::lock_guard<std::mutex> lk(g_pin_mu);
    if (std::find(g_bar_absent.begin(), g_bar_absent.end(), device) != g_bar_absent.end()) return nullptr;
    for (size_t i = 0; i < g_bar_free.size(); ++i)
      if (std::get<0>(g_bar_free[i]) == device && std::get<1>(g_bar_free[i]) >= bytes) {
        bytes = std::get<1>(g_bar_free[i]);
        p = std::get<2>(g_bar_free[i]);
        g_bar_free.erase(g_bar_free.begin() + (long)i);
        break;
      }
  }
  if (!p) {
    if (hipExtMallocWithFlags(&p, bytes, hipDeviceMallocFinegrained) != hipSuccess) {
      (void)hipGetLastError();
      return nullptr;  // (this engine only: an allocation failure may be transient)
    }
    if (!host_mapped(p, bytes)) {  // the host cannot map this device's memory: for the whole process
      std::lock_guard<std::mutex> lk(g_pin_mu);
      g_bar_absent.push_back(device);
      g_bar_free.emplace_back(device, bytes, p);  // (kept: hipFree would synchronise the device)
      return nullptr;
    }
  }
  std::memset(p, 0, bytes);  // (through the mapping: a reused ring holds another engine's tags)
  _mm_sfence();
  return p;
}

void bar_give(int device, void *p, size_t bytes) {
  std::lock_guard<std::mutex> lk(g_pin_mu);
  g_bar_free.emplace_back(device, bytes, p);
}

// Every entry point leaves the calling thread's current HIP device as it found it
// (the engine switches to its own device for its work).
struct DeviceRestore {
  int prev = -1;
  DeviceRestore() {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
  }
  ~DeviceRestore() {
    int cur = -1;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
};

}  // namespace

namespace {
void res_register(go2pi_engine *e);
unsigned *yield_word(int device);
void res_unregister(go2pi_engine *e);
std::unique_lock<std::mutex> evict_residents(const go2pi_engine *self, int64_t batch);
// The process-wide registry of engines that may hold a resident kernel, and the lock
// that orders a batched launch's eviction + enqueue against every resident relaunch
// (evict_residents, resident_start)
std::mutex g_res_mu;
}  // namespace

struct go2pi_engine {
  go2pi::Model model;
  go2pi_opts opts{};
  int device = 0;
  int waves = 8;
  int small_batch = 8;
  hipStream_t stream = nullptr;
  go2pi::DevProgram prog{};
  std::vector<void *> allocs;  // device allocations
  std::vector<std::pair<size_t, void *>> pinned;  // pinned host blocks (returned to the cache)
  float *d_hidden = nullptr;   // [max_batch][H]
  float *d_obs = nullptr;      // host-path staging [max_batch][in]
  float *d_act = nullptr;      // [max_batch][out]
  float *d_tmp[2] = {nullptr, nullptr};  // small-batch activations [SMALL_MAXB][maxw]
  int tmp_stride = 0;
  float *h_obs = nullptr, *h_act = nullptr;  // pinned, host-mapped
  float *m_obs = nullptr, *m_act = nullptr;  // device aliases of the above
  unsigned long long *h_actg = nullptr, *m_actg = nullptr;  // resident act(): {epoch, value} action granules
  size_t n_actg = 0;
  hipGraphExec_t graphs[GO2PI_SMALL_MAXB + 1] = {};
  hipGraph_t graph_defs[GO2PI_SMALL_MAXB + 1] = {};
  go2pi_cost cost{};
  int64_t n_stamps = 0;
  // single-launch small-batch path (policy_latency_kernel)
  bool latency_ok = false;
  unsigned long long *d_gran = nullptr;  // [nl-1][gstride] {tag, value} granules
  int gstride = 0;
  unsigned *h_err = nullptr, *m_err = nullptr;    // host-mapped error words: [0] batch-1 hand-off, [64] batched
                                                   // kernel layer hand-off (each on its own cache line)
  unsigned *h_done = nullptr, *m_done = nullptr;  // host-mapped completion word (own cache line)
  bool done_ok = false;                            // final layer is one tile: WG 0 signals completion
  go2pi::DevProgram *d_prog = nullptr;             // device copy of prog (what every kernel reads)
  unsigned epoch = 1, last_epoch = 0;
  // resident batch <= SMALL_MAXB path (resident.hip, opts.resident_ms > 0)
  bool resident_ok = false, resident_live = false;
  std::atomic<int> res_flag{0};  // resident_live, readable from other threads (evict_residents)
  bool resident_ctl_ok = false;  // the controller-tick form applies (dense policies)
  unsigned long long *d_hgran = nullptr;  // GRU form: [2][SMALL_MAXB][H] hidden-row granules (two buffers)
  bool resident_ctl = false;  // the live kernel is the controller-tick form
  bool resident1 = false;     // act() form in one workgroup (resident.hip policy_resident1_kernel)
  bool resident1_ctl = false; // controller form in one workgroup (512 threads)
  bool wide = false;          // act() form for wide policies (resident_wide.hip policy_wide_kernel, r06)
  int64_t res_launches = 0;   // resident kernel launches (go2pi_resident_launches)
  bool ctl_gran_ok = false;   // ... answered in granules (policy_act1_kernel, r05): no done word per tick
  std::vector<float> res_rows = std::vector<float>(GO2PI_SMALL_MAXB * (GO2PI_CTL_RAW + 16 * GO2PI_CTL_STEP_DIM));
  unsigned long long *h_req = nullptr, *m_req = nullptr;  // request granules: host view, device view
  size_t req_bar_bytes = 0;  // > 0: the ring is in device memory the host writes through the BAR (bar_take)
  unsigned long long *d_mirror = nullptr;                 // device copy of the request (workgroup 0 -> the rest)
  unsigned long long res_idle_ticks = 0;                  // 100 MHz wall-clock ticks
  std::chrono::steady_clock::time_point res_last{};
  // controller tick (go2pi_controller_step*)
  int ctl_hist = 0;                        // kHistory when the policy's I/O is a Go2 controller's, else 0
  go2pi::DevCtlParams *d_ctl = nullptr;    // device copy of the parameters
  char *h_ctl = nullptr, *m_ctl = nullptr; // host path, batch <= SMALL_MAXB: pinned host-mapped staging
  char *d_ctlbuf = nullptr;                // host path, larger batches: device staging (lazy)

  // Teardown touches only this engine's stream: no hipFree / hipHostFree /
  // hipDeviceSynchronize, each of which would wait for every other engine's live
  // resident kernel on the device (device memory is stream-ordered, pinned
  // blocks go back to the process-wide cache).
  ~go2pi_engine() {
    DeviceRestore keep;
    if (resident_ok) res_unregister(this);
    (void)hipSetDevice(device);
    if (resident_live) {  // tell the resident kernel to leave (the sync below waits for it)
      __atomic_store_n(h_req, (unsigned long long)GO2PI_RES_LEAVE << 32, __ATOMIC_SEQ_CST);
      resident_live = false;
    }
    if (stream) (void)hipStreamSynchronize(stream);
    for (int i = 0; i <= GO2PI_SMALL_MAXB; ++i) {
      if (graphs[i]) (void)hipGraphExecDestroy(graphs[i]);
      if (graph_defs[i]) (void)hipGraphDestroy(graph_defs[i]);
    }
    for (void *p : allocs) (void)hipFreeAsync(p, stream);
    for (auto &b : pinned) pin_give(b.second, b.first);
    if (req_bar_bytes) bar_give(device, h_req, req_bar_bytes);
    if (stream) {
      (void)hipStreamSynchronize(stream);
      (void)hipStreamDestroy(stream);
    }
  }

  // device memory: stream-ordered on the engine's stream (usable by any stream once
  // dalloc returns)
  template <class T>
  T *dalloc(size_t count) {
    void *p = nullptr;
    hip_check(hipMallocAsync(&p, std::max<size_t>(count, 1) * sizeof(T), stream), "hipMallocAsync");
    allocs.push_back(p);
    hip_check(hipStreamSynchronize(stream), "hipStreamSynchronize");
    return static_cast<T *>(p);
  }
  // pinned, host-mapped (fine-grained) memory and its device alias
  template <class T>
  void palloc(T **host, T **dev, size_t bytes) {
    size_t got = bytes;
    void *p = pin_take(got);
    pinned.emplace_back(got, p);  // the block's real size goes back to the cache
    std::memset(p, 0, bytes);
    *host = static_cast<T *>(p);
    if (dev) hip_check(hipHostGetDevicePointer((void **)dev, p, 0), "hipHostGetDevicePointer");
  }
  template <class T>
  T *upload(const std::vector<T> &v) {
    T *p = dalloc<T>(v.size());
    if (!v.empty()) hip_check(hipMemcpy(p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice), "hipMemcpy");
    return p;
  }

  bool use_chain(int64_t batch) const {
    return !model.has_gru && small_batch > 0 && batch <= small_batch;
  }

  bool use_latency(int64_t batch) const { return latency_ok && batch <= GO2PI_SMALL_MAXB; }

  // Enqueue one forward over `batch` rows (obs/act: device-accessible pointers).
  // done (single-launch path only): host-mapped word the kernel sets to the call's epoch.
  // granule tags of the next single-launch call (layer l of this call: e0 + l)
  unsigned next_epoch(hipStream_t s) {
    const unsigned n = (unsigned)prog.nl;
    if (epoch > 0xFFFFFFFFu - 2 * n) {  // tag space exhausted (~1e9 calls): clear granules, restart
      hip_check(hipMemsetAsync(d_gran, 0, sizeof(unsigned long long) * (size_t)(prog.nl - 1) * gstride, s),
                "hipMemsetAsync");
      epoch = 1;
    }
    const unsigned e0 = epoch;
    epoch += n;
    last_epoch = e0;
    return e0;
  }

  // Host spin on the host-mapped completion word of the single-launch path;
  // false: not observed within 2 s (the caller falls back to a stream sync).
  bool spin_done() {
    const unsigned want = last_epoch;
    const auto t0 = std::chrono::steady_clock::now();
    for (unsigned it = 0; __atomic_load_n(h_done, __ATOMIC_ACQUIRE) != want; ++it) {
      __builtin_ia32_pause();
      if ((it & 1023) == 1023 && std::chrono::steady_clock::now() - t0 > std::chrono::seconds(2)) break;
    }
    return __atomic_load_n(h_done, __ATOMIC_ACQUIRE) == want;
  }

  // ---- resident path: one launch serves every batch <= SMALL_MAXB go2pi_run
  // until another call needs the stream (resident_stop) or it idles out.
  void resident_stop() {
    if (!resident_live) return;
    __atomic_store_n(h_req, (unsigned long long)GO2PI_RES_LEAVE << 32, __ATOMIC_SEQ_CST);
    resident_live = false;
    res_flag.store(0);
    hip_check(hipStreamSynchronize(stream), "hipStreamSynchronize (resident kernel leaving)");
  }
  void resident_start(const go2pi::DevCtl *ctl) {
    // (never between another thread's eviction and its batched launch: evict_residents)
    std::lock_guard<std::mutex> res_lk(g_res_mu);
    const size_t ng = (size_t)std::max(1, prog.nl - 1) * gstride;
    hip_check(hipMemsetAsync(d_gran, 0, ng * sizeof(unsigned long long), stream), "hipMemsetAsync");
    hip_check(hipMemsetAsync(d_mirror, 0, sizeof(unsigned long long) * (1 + GO2PI_SMALL_MAXB * (size_t)model.in_dim),
                             stream),
              "hipMemsetAsync");
    if (d_hgran)
      hip_check(hipMemsetAsync(d_hgran, 0, sizeof(unsigned long long) * 2 * GO2PI_SMALL_MAXB * (size_t)model.gru.H,
                               stream),
                "hipMemsetAsync");
    __atomic_store_n(h_req, 0ull, __ATOMIC_SEQ_CST);
    __atomic_store_n(h_done, 0u, __ATOMIC_SEQ_CST);
    std::memset(h_actg, 0, sizeof(unsigned long long) * n_actg);
    if (ctl ? resident1_ctl : resident1)
      hip_check(go2pi::launch_resident1(prog, d_prog, m_req, m_actg, m_err, m_done, res_idle_ticks, prog.yield, ctl,
                                        stream),
                "resident launch (one workgroup)");
    else if (!ctl && wide)
      hip_check(go2pi::launch_resident_wide(prog, d_prog, m_req, m_actg, d_gran, gstride, m_err, m_done, res_idle_ticks,
                                            prog.yield, stream),
                "resident launch (wide policy)");
    else
      hip_check(go2pi::launch_resident(prog, d_prog, m_req, m_actg, d_gran, gstride, d_mirror, m_err, m_done,
                                       res_idle_ticks, ctl, d_hgran, d_hidden, prog.yield, stream),
                "resident launch");
    ++res_launches;
    resident_live = true;
    res_flag.store(1);
    resident_ctl = ctl != nullptr;
    res_last = std::chrono::steady_clock::now();
  }
  // One request to the resident kernel. ctl null: act(), `rows` = obs [batch][in_dim];
  // the action lands in h_act. ctl: a controller tick, `rows` = its inputs concatenated
  // (state | joystick | obs | action, each batch rows); the outputs land in the staging
  // ctl names; flags = GO2PI_RES_* bits. The rows travel as tagged granules.
  // false: not served because the kernel kept being told to leave (a batched launch
  // on the device evicts live resident kernels, evict_residents): the caller serves
  // the request by a launch instead; the kernel is relaunched by a later call.
  // go2pi_run's fast path makes no HIP call while a live kernel serves it (lazy_dev):
  // need_device() switches the calling thread to the engine's device the first time a
  // stop or relaunch needs the runtime, and dev_done() switches it back.
  bool lazy_dev = false, dev_switched = false;
  int dev_saved = -1;
  void need_device() {
    if (!lazy_dev || dev_switched) return;
    if (hipGetDevice(&dev_saved) != hipSuccess) dev_saved = -1;
    hip_check(hipSetDevice(device), "hipSetDevice");
    dev_switched = true;
  }
  void dev_done() {
    if (dev_switched && dev_saved >= 0 && dev_saved != device) (void)hipSetDevice(dev_saved);
    lazy_dev = dev_switched = false;
  }
  // the live kernel serves the next request as it is (no stop or relaunch due first)
  bool resident_ready(const go2pi::DevCtl *ctl) const {
    const auto idle = std::chrono::microseconds(1000LL * opts.resident_ms);
    return resident_live && resident_ctl == (ctl != nullptr) && std::chrono::steady_clock::now() - res_last <= idle / 2 &&
           __atomic_load_n(h_done, __ATOMIC_ACQUIRE) != GO2PI_RES_LEAVE &&
           epoch <= 0xFFFFFFF0u - 2 * ((unsigned)prog.nl + 2);
  }
  // The granules of one request's answer: {offset, count} ranges of h_actg (act(): the
  // action rows; the controller form's: the requested outputs, the observation rows
  // first, as the kernel stores them first). The scan resumes where it stopped.
  struct GranScan {
    int r[6][2];
    int nr = 0, ri = 0, k = 0;
    void add(int off, int n) {
      r[nr][0] = off;
      r[nr++][1] = n;
    }
  };
  GranScan gran_scan(bool ctl, int64_t batch, unsigned flags) const {
    GranScan sc;
    const int b = (int)batch;
    if (!ctl) {
      sc.add(0, b * model.out_dim);
      return sc;
    }
    const go2pi::CtlGran G = go2pi::ctl_gran(model.in_dim);
    sc.add(G.obs, b * model.in_dim);
    if (flags & GO2PI_RES_STATUS) sc.add(G.status, b);
    sc.add(G.act, b * GO2PI_CTL_DOF);
    if (flags & GO2PI_RES_QDES) sc.add(G.qdes, 2 * b * GO2PI_CTL_DOF);
    if (flags & GO2PI_RES_KP) sc.add(G.kp, 2 * b * GO2PI_CTL_DOF);
    if (flags & GO2PI_RES_KD) sc.add(G.kd, 2 * b * GO2PI_CTL_DOF);
    return sc;
  }
  // true once every granule of sc carries tag e0
  bool gran_done(GranScan &sc, unsigned e0) const {
    for (; sc.ri < sc.nr; ++sc.ri, sc.k = 0) {
      const unsigned long long *g = h_actg + sc.r[sc.ri][0];
      const int n = sc.r[sc.ri][1];
      while (sc.k < n && (unsigned)(__atomic_load_n(g + sc.k, __ATOMIC_ACQUIRE) >> 32) == e0) ++sc.k;
      if (sc.k < n) return false;
    }
    return true;
  }
  // the act() answer's values to h_act
  void act_take(int64_t batch) {
    const int nout = (int)batch * model.out_dim;
    for (int j = 0; j < nout; ++j) {
      const unsigned bits = (unsigned)__atomic_load_n(h_actg + j, __ATOMIC_RELAXED);
      std::memcpy(h_act + j, &bits, 4);
    }
  }
  // the controller form's answer granules to the caller's buffers (ctl_gran_ok)
  void ctl_take(int64_t batch, float *obs, float *action, double *q_des, double *kp, double *kd,
                uint32_t *status) const {
    const go2pi::CtlGran G = go2pi::ctl_gran(model.in_dim);
    const int b = (int)batch, nd = b * GO2PI_CTL_DOF;
    auto lo = [&](int i) { return (uint32_t)__atomic_load_n(h_actg + i, __ATOMIC_RELAXED); };
    auto f64 = [&](int off, double *dst) {
      for (int i = 0; i < nd; ++i) {
        const uint64_t bits = (uint64_t)lo(off + 2 * i) | ((uint64_t)lo(off + 2 * i + 1) << 32);
        std::memcpy(dst + i, &bits, 8);
      }
    };
    for (int i = 0; i < b * model.in_dim; ++i) {
      const uint32_t bits = lo(G.obs + i);
      std::memcpy(obs + i, &bits, 4);
    }
    for (int i = 0; i < nd; ++i) {
      const uint32_t bits = lo(G.act + i);
      std::memcpy(action + i, &bits, 4);
    }
    if (q_des) f64(G.qdes, q_des);
    if (kp) f64(G.kp, kp);
    if (kd) f64(G.kd, kd);
    if (status)
      for (int i = 0; i < b; ++i) status[i] = lo(G.status + i);
  }
  bool resident_serve(const go2pi::DevCtl *ctl, const float *rows, int64_t batch, unsigned flags) {
    if (resident_live && resident_ctl != (ctl != nullptr)) {  // the other form is live
      need_device();
      resident_stop();
    }
    const int n = (int)batch * (model.in_dim + (ctl ? GO2PI_CTL_RAW : 0));
    const auto idle = std::chrono::microseconds(1000LL * opts.resident_ms);  // (us: idle / 2 stays > 0 at 1 ms)
    for (int attempt = 0;; ++attempt) {
      // layer tags e + 1 + l: an epoch spans nl + 2 tags
      const unsigned span = (unsigned)prog.nl + 2;
      if (epoch > 0xFFFFFFF0u - 2 * span) {  // tag space exhausted: restart with zeroed granules
        need_device();
        resident_stop();
        epoch = 1;
      }
      const unsigned e0 = epoch;
      epoch += span;
      last_epoch = e0;
      const auto now = std::chrono::steady_clock::now();
      // the kernel leaves after resident_ms idle: past half of it, relaunch rather than race its exit
      if (resident_live && (now - res_last > idle / 2 || __atomic_load_n(h_done, __ATOMIC_ACQUIRE) == GO2PI_RES_LEAVE)) {
        need_device();
        resident_stop();
      }
      if (!resident_live) {
        need_device();
        resident_start(ctl);
      }
      for (int i = 0; i < n; ++i) {
        unsigned bits;
        std::memcpy(&bits, rows + i, 4);
        __atomic_store_n(h_req + 1 + i, ((unsigned long long)e0 << 32) | bits, __ATOMIC_RELAXED);
      }
      __atomic_store_n(h_req, ((unsigned long long)e0 << 32) | (unsigned)batch | flags, __ATOMIC_RELEASE);
      if (req_bar_bytes) _mm_sfence();  // the BAR mapping is write-combined: send the request now
      const auto t0 = std::chrono::steady_clock::now();
      unsigned d;
      // act() and the granule controller form: the answer granules themselves, every tag =
      // this request's epoch; the r04 / multi-workgroup controller forms: a done word
      // behind the drained outputs
      const bool gran = !ctl || ctl_gran_ok;
      if (!gran) {
        for (unsigned it = 0; (d = __atomic_load_n(h_done, __ATOMIC_ACQUIRE)) != e0 && d != GO2PI_RES_LEAVE; ++it) {
          __builtin_ia32_pause();
          if ((it & 1023) == 1023 && std::chrono::steady_clock::now() - t0 > std::chrono::seconds(2)) break;
        }
      } else {
        GranScan sc = gran_scan(ctl != nullptr, batch, flags);
        for (unsigned it = 0;; ++it) {
          if (gran_done(sc, e0)) {
            d = e0;
            break;
          }
          if ((d = __atomic_load_n(h_done, __ATOMIC_ACQUIRE)) == GO2PI_RES_LEAVE) {
            // the kernel may have answered this request and then left (a LEAVE header
            // from evict_residents, or a moved yield counter): its answer granules are
            // acknowledged before the LEAVE done word (resident.hip: vmcnt(0), barrier,
            // then done), so a rescan after seeing LEAVE finds them if it served the
            // request. Treating a served request as unserved would run it twice: for a
            // GRU / LSTM policy, advancing the hidden state twice.
            GranScan again = gran_scan(ctl != nullptr, batch, flags);
            if (gran_done(again, e0)) d = e0;
            break;
          }
          __builtin_ia32_pause();
          if ((it & 1023) == 1023 && std::chrono::steady_clock::now() - t0 > std::chrono::seconds(2)) break;
        }
        if (d == e0 && !ctl) act_take(batch);
      }
      res_last = std::chrono::steady_clock::now();
      if (d == e0) return true;
      // the kernel left: wait for it to drain. An idle exit racing this request is
      // benign (serve it from a fresh launch with a fresh epoch); a hand-off timeout
      // (h_err set) is a device-side protocol fault and is reported, not retried
      need_device();
      resident_stop();
      if (gran) {  // the kernel has exited (stream synced): a request it served has every granule
        GranScan again = gran_scan(ctl != nullptr, batch, flags);
        if (gran_done(again, e0)) {
          if (!ctl) act_take(batch);
          return true;
        }
      }
      if (__atomic_load_n(h_err, __ATOMIC_ACQUIRE)) {
        __atomic_store_n(h_err, 0u, __ATOMIC_RELEASE);
        throw HipError("resident kernel: a layer hand-off timed out (request not served)", GO2PI_E_DEVICE);
      }
      if (d != GO2PI_RES_LEAVE)
        throw HipError("resident kernel did not answer within 2 s (request not served)", GO2PI_E_DEVICE);
      if (attempt >= 1) return false;  // evicted again (or idle exit twice): serve by a launch
    }
  }

  void check_handoff() {
    if (h_err && __atomic_load_n(h_err, __ATOMIC_ACQUIRE)) {
      __atomic_store_n(h_err, 0u, __ATOMIC_RELEASE);
      throw HipError("batch-1 kernel hand-off timed out (workgroups not co-resident?)", GO2PI_E_DEVICE);
    }
    if (h_err && __atomic_load_n(h_err + 64, __ATOMIC_ACQUIRE)) {
      __atomic_store_n(h_err + 64, 0u, __ATOMIC_RELEASE);
      throw HipError("batched kernel: a layer hand-off between waves timed out (outputs invalid)", GO2PI_E_DEVICE);
    }
  }

  // Enqueue one controller tick (device-accessible pointers in c).
  void enqueue_ctl(const go2pi::DevCtl &c, int64_t batch, hipStream_t s, unsigned *done = nullptr) {
    if (use_latency(batch) && done_ok) {
      const unsigned e0 = next_epoch(s);
      hip_check(go2pi::launch_latency_ctl(prog, d_prog, c, (int)batch, e0, d_gran, gstride, m_err, done, s),
                "controller latency launch");
    } else {
      hip_check(go2pi::launch_policy_fused_ctl(prog, d_prog, waves, c, d_hidden, (int)batch, s),
                "controller fused launch");
    }
  }

  void enqueue(const float *obs, float *act, int64_t batch, hipStream_t s, unsigned *done = nullptr) {
    if (use_latency(batch)) {
      const unsigned e0 = next_epoch(s);
      hip_check(go2pi::launch_latency(prog, d_prog, obs, act, (int)batch, e0, d_gran, gstride, m_err, done, s),
                "latency launch");
    } else if (use_chain(batch)) {
      const float *x = obs;
      int xs = prog.in_dim;
      for (int l = 0; l < prog.nl; ++l) {
        const bool last = l == prog.nl - 1;
        float *y = last ? act : d_tmp[l & 1];
        const int ys = last ? prog.out_dim : tmp_stride;
        hip_check(go2pi::launch_gemv_layer(prog, l, x, xs, y, ys, (int)batch, s), "gemv_layer launch");
        x = y;
        xs = ys;
      }
    } else {
      hip_check(go2pi::launch_policy_fused(prog, d_prog, waves, obs, act, d_hidden, (int)batch, 1, s), "fused launch");
    }
  }

  hipGraphExec_t graph_for(int b) {
    if (graphs[b]) return graphs[b];
    hip_check(hipStreamBeginCapture(stream, hipStreamCaptureModeThreadLocal), "hipStreamBeginCapture");
    try {
      enqueue(m_obs, m_act, b, stream);
    } catch (...) {
      hipGraph_t g = nullptr;
      (void)hipStreamEndCapture(stream, &g);
      if (g) (void)hipGraphDestroy(g);
      throw;
    }
    hip_check(hipStreamEndCapture(stream, &graph_defs[b]), "hipStreamEndCapture");
    hip_check(hipGraphInstantiate(&graphs[b], graph_defs[b], nullptr, nullptr, 0), "hipGraphInstantiate");
    return graphs[b];
  }
};

namespace {

// Live resident kernels of every engine in the process, by device. A resident
// kernel holds its workgroups' CUs while it waits for requests; a batched launch
// (which wants all 256 CUs, one workgroup each) on the same device then runs in two
// rounds: measured 37.8 -> 71.4 us per 4096-robot step (tools/interference.py,
// DESIGN §4.2b). So every batched launch first tells the other engines' live
// resident kernels on its device to leave (a LEAVE header; no wait), and their
// next act() relaunches.
std::vector<go2pi_engine *> g_res_engines;

void res_register(go2pi_engine *e) {
  std::lock_guard<std::mutex> lk(g_res_mu);
  g_res_engines.push_back(e);
}

void res_unregister(go2pi_engine *e) {
  std::lock_guard<std::mutex> lk(g_res_mu);
  g_res_engines.erase(std::remove(g_res_engines.begin(), g_res_engines.end(), e), g_res_engines.end());
}

// The batched-launch counter of each device (DevProgram::yield), one per process
// and device, never freed (hipFree would synchronise the device).
unsigned *yield_word(int device) {
  static std::mutex mu;
  static std::vector<unsigned *> words;
  std::lock_guard<std::mutex> lk(mu);
  if ((int)words.size() <= device) words.resize(device + 1, nullptr);
  if (!words[device]) {
    void *p = nullptr;
    hip_check(hipMalloc(&p, 256), "hipMalloc");
    hip_check(hipMemset(p, 0, 256), "hipMemset");
    words[device] = static_cast<unsigned *>(p);
  }
  return words[device];
}

// batch: the rows of the launch that follows (one 16-row workgroup each); a launch of
// at most GO2PI_YIELD_MIN_GRID workgroups fits beside the resident kernels and evicts
// none (the kernels' own yield bump has the same bound, program.hpp).
// The lock comes back held: the caller keeps it until its batched launch is enqueued.
// A resident kernel another thread relaunched in between (resident_start takes the same
// lock) could otherwise sit ahead of that launch in a hardware queue two streams share,
// and serve its own requests until it idles out while the launch waits behind it (it
// leaves on the launch's yield bump only once the launch has started).
std::unique_lock<std::mutex> evict_residents(const go2pi_engine *self, int64_t batch) {
  if ((batch + GO2PI_TILE_ROWS - 1) / GO2PI_TILE_ROWS <= GO2PI_YIELD_MIN_GRID) return {};
  std::unique_lock<std::mutex> lk(g_res_mu);
  for (go2pi_engine *o : g_res_engines)
    if (o != self && o->device == self->device && o->res_flag.load() == 1)
      __atomic_store_n(o->h_req, (unsigned long long)GO2PI_RES_LEAVE << 32, __ATOMIC_SEQ_CST);
  return lk;
}

// K is padded to a multiple of 64 (4 chunks: the kernel's unroll); a hidden layer's
// N to its consumer's K_pad (64), the final layer's N to 16 (one MFMA tile).
void pack_dense(const go2pi::Dense &d, bool last, std::vector<float> &w, std::vector<float> &b, int &K_pad,
                int &N_pad, int kq = 64) {
  K_pad = kq == 16 ? ceil16(d.K) : ceil64(d.K);
  N_pad = last ? ceil16(d.N) : ceil64(d.N);
  const int T = N_pad / 16, C = K_pad / 16;
  w.assign((size_t)T * C * 64 * 4, 0.f);
  for (int t = 0; t < T; ++t)
    for (int c = 0; c < C; ++c)
      for (int lane = 0; lane < 64; ++lane)
        for (int j = 0; j < 4; ++j) {
          const int n = 16 * t + (lane & 15), k = 16 * c + 4 * (lane >> 4) + j;
          w[(((size_t)c * T + t) * 64 + lane) * 4 + j] = (n < d.N && k < d.K) ? d.W[(size_t)n * d.K + k] : 0.f;
        }
  b.assign(N_pad, 0.f);
  std::copy(d.b.begin(), d.b.end(), b.begin());
}

// Recurrent-cell fragments: [Cx + Ch][Ht][gate][lane] float4 over the concatenated
// [x (I_pad) | h (H)] axis; x chunks carry W, h chunks carry R. G = 3 gates (GRU:
// z, r, h) or 4 (LSTM: i, o, f, c), in ONNX row order.
void pack_gru(const go2pi::Gru &g, std::vector<float> &w, int &I_pad) {
  I_pad = ceil64(g.I);  // whole 4-chunk groups of x (the pipelined cell's ring runs on them)
  const int H = g.H, Ht = H / 16, Cx = I_pad / 16, Ch = H / 16, Cc = Cx + Ch, G = g.G;
  w.assign((size_t)Ht * Cc * G * 64 * 4, 0.f);
  for (int t = 0; t < Ht; ++t)
    for (int c = 0; c < Cc; ++c)
      for (int gate = 0; gate < G; ++gate)
        for (int lane = 0; lane < 64; ++lane)
          for (int j = 0; j < 4; ++j) {
            const int unit = 16 * t + (lane & 15);
            const int row = gate * H + unit;
            float v = 0.f;
            if (c < Cx) {
              const int k = 16 * c + 4 * (lane >> 4) + j;
              if (k < g.I) v = g.W[(size_t)row * g.I + k];
            } else {
              const int k = 16 * (c - Cx) + 4 * (lane >> 4) + j;
              v = g.R[(size_t)row * H + k];
            }
            w[((((size_t)c * Ht + t) * G + gate) * 64 + lane) * 4 + j] = v;
          }
}

void set_ctl_params(go2pi_engine &e, const go2pi_ctl_params &cp) {
  go2pi::DevCtlParams d{};
  for (int i = 0; i < GO2PI_CTL_DOF; ++i) d.q0[i] = cp.q0[i];
  d.action_scale = cp.action_scale;
  d.kp_run = (double)cp.kp;  // float members widened at send_command (controller.cpp:246-247)
  d.kd_run = (double)cp.kd;
  d.kp_stop = (double)cp.kp_stop;
  d.action_limit = cp.action_limit;
  d.contact_threshold = cp.contact_threshold;
  for (int i = 0; i < 3; ++i) d.gravity_w[i] = cp.gravity_w[i];
  d.hist = e.ctl_hist;
  hip_check(hipMemcpy(e.d_ctl, &d, sizeof(d), hipMemcpyHostToDevice), "hipMemcpy");
}

// The 4-wave uniform-MLP pipeline (fused_impl.hpp w4_step) applies to a policy
// whose hidden layers are all 64 * TPW wide (TPW = 2, 4 or 8) with one
// activation, and whose final layer is at most 2 tiles wide (1 at TPW = 8); a GRU
// in front needs H % 64 == 0. It is the default (waves = 0) wherever it applies:
// measured faster than the generic 8-wave body.
bool w4_eligible(const go2pi_engine &e, const go2pi::Model &m) {
  const int nl = (int)m.layers.size();
  if (!(e.opts.waves == 0 || e.opts.waves == 4) || nl < 2) return false;
  if (m.has_gru && m.gru.H % 64) return false;
  if (m.has_gru && m.gru.cell == 0 && m.gru.lbr == 0) return false;  // the two-pass cell: generic body only
  if (std::getenv("GO2PI_NO_HEAD_FUSE") || std::getenv("GO2PI_NO_W4")) return false;  // env: A/B diagnostics only
  const int tpw = ceil64(m.layers[0].N) / 64, t_last = ceil16(m.layers[nl - 1].N) / 16;
  if (!(tpw == 2 || tpw == 4 || tpw == 8) || t_last > (tpw == 8 ? 1 : 2)) return false;
  for (int l = 0; l + 1 < nl; ++l)
    if (ceil64(m.layers[l].N) != 64 * tpw || m.layers[l].act != m.layers[0].act ||
        m.layers[l].alpha != m.layers[0].alpha || m.layers[l].beta != m.layers[0].beta)
      return false;
  return true;
}

void build(go2pi_engine &e, const uint8_t *bytes, size_t n, const go2pi_opts *o) {
  go2pi_default_opts(&e.opts);
  if (o) {
    if (o->struct_size < (int32_t)offsetof(go2pi_opts, obs_mean))
      throw ApiError("go2pi_opts.struct_size too small", GO2PI_E_INVALID);
    std::memcpy(&e.opts, o, std::min<size_t>(sizeof(go2pi_opts), (size_t)o->struct_size));
    e.opts.struct_size = sizeof(go2pi_opts);
  }
  if (e.opts.max_batch <= 0) e.opts.max_batch = 4096;
  if (e.opts.max_batch > (int64_t)std::numeric_limits<int>::max() / 2)
    throw ApiError("max_batch too large", GO2PI_E_INVALID);
  try {
    e.model = go2pi::parse_onnx(bytes, n);
  } catch (const std::exception &ex) {
    throw ApiError(ex.what(), GO2PI_E_MODEL);
  }
  auto &m = e.model;
  if ((int)m.layers.size() > GO2PI_MAX_LAYERS)
    throw ApiError("policy has more than " + std::to_string(GO2PI_MAX_LAYERS) + " dense layers", GO2PI_E_MODEL);
  if (m.has_gru) {
    // lbr = 0 (Keras reset_after=False) runs the generic body's two-pass cell
    // (fused_impl.hpp gru0_cell), one tile group per wave: H <= 256
    if (m.gru.cell == 0 && m.gru.lbr == 0 && m.gru.H > 256)
      throw ApiError("GRU linear_before_reset=0 with hidden size > 256 is not supported", GO2PI_E_MODEL);
    if (m.gru.H % 16) throw ApiError("recurrent hidden size must be a multiple of 16", GO2PI_E_MODEL);
  }

  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
    throw ApiError("no HIP device available (go2pi has no CPU fallback)", GO2PI_E_DEVICE);
  if (e.opts.device < 0 || e.opts.device >= ndev)
    throw ApiError("device ordinal " + std::to_string(e.opts.device) + " out of range", GO2PI_E_INVALID);
  e.device = e.opts.device;
  hip_check(hipSetDevice(e.device), "hipSetDevice");
  hip_check(hipStreamCreateWithFlags(&e.stream, hipStreamNonBlocking), "hipStreamCreate");

  // 8 waves per 16-robot workgroup (2 per SIMD) measured fastest with the
  // interleaved schedule (kernels.hip, dense_acc note): 104K vs 106K cycles at 16
  e.waves = (e.opts.waves == 4 || e.opts.waves == 16) ? e.opts.waves : 8;
  e.small_batch = e.opts.small_batch == 0 ? GO2PI_SMALL_MAXB : std::min<int>(e.opts.small_batch, GO2PI_SMALL_MAXB);

  go2pi::DevProgram &p = e.prog;
  std::memset(&p, 0, sizeof(p));
  p.nl = (int)m.layers.size();
  p.in_dim = m.in_dim;
  p.out_dim = m.out_dim;
  int maxw = 0;
  double flops = 0, wbytes = 0;
  // The 4-wave pipeline (decided below) takes a layer 0 of 3 (mod 4) k-chunks:
  // a 48- or 98-wide observation is padded to 16 columns, not 64 (25 % / 12.5 %
  // fewer layer-0 MFMAs and fragment bytes). Other kernels take any chunk count.
  const bool w4_shape = w4_eligible(e, m);
  const int k0q = (w4_shape && !m.has_gru && (ceil16(m.layers[0].K) / 16) % 4 == 3 && !std::getenv("GO2PI_K0_PAD64"))
                      ? 16 : 64;  // env: A/B diagnostics only
  // every dense layer's fragments back to back in one arena (the pipeline finds
  // layer l from the base: fused_impl.hpp w4_layer_w)
  std::vector<std::vector<float>> packed(p.nl);
  size_t arena = 0;
  std::vector<size_t> off(p.nl);
  for (int l = 0; l < p.nl; ++l) {
    std::vector<float> b;
    int kp, np;
    pack_dense(m.layers[l], l == p.nl - 1, packed[l], b, kp, np, l == 0 ? k0q : 64);
    off[l] = arena;
    arena += packed[l].size();
    auto &L = p.L[l];
    L.bias = e.upload(b);
    L.K_pad = kp;
    L.N_pad = np;
    L.N = m.layers[l].N;
    L.act = m.layers[l].act;
    L.alpha = m.layers[l].alpha;
    L.beta = m.layers[l].beta;
    maxw = std::max({maxw, kp, np});
    flops += 2.0 * m.layers[l].K * m.layers[l].N;
    wbytes += 4.0 * ((double)m.layers[l].K * m.layers[l].N + m.layers[l].N);
  }
  {
    std::vector<float> all;
    all.reserve(arena);
    for (auto &v : packed) all.insert(all.end(), v.begin(), v.end());
    const float *base = e.upload(all);
    for (int l = 0; l < p.nl; ++l) p.L[l].w = base + off[l];
  }
  if (m.has_gru) {
    std::vector<float> w;
    int ip;
    pack_gru(m.gru, w, ip);
    const int H = m.gru.H, G = m.gru.G;
    std::vector<float> bzr(2 * H), bh(2 * H);
    if (m.gru.cell == 1) {  // LSTM: every gate's two biases summed (i, o, f, c)
      bzr.resize(4 * H);
      for (int j = 0; j < 4 * H; ++j) bzr[j] = m.gru.Wb[j] + m.gru.Rb[j];
    } else {
      for (int j = 0; j < H; ++j) {
        bzr[j] = m.gru.Wb[j] + m.gru.Rb[j];
        bzr[H + j] = m.gru.Wb[H + j] + m.gru.Rb[H + j];
        bh[j] = m.gru.Wb[2 * H + j];
        bh[H + j] = m.gru.Rb[2 * H + j];
      }
    }
    p.has_gru = 1;
    p.gru.w = e.upload(w);
    p.gru.bzr = e.upload(bzr);
    p.gru.bh = e.upload(bh);
    p.gru.I = m.gru.I;
    p.gru.I_pad = ip;
    p.gru.H = H;
    p.gru.lbr = m.gru.lbr;
    p.gru.cell = m.gru.cell;
    p.gru.sw = m.gru.cell == 1 ? 2 * H : H;
    p.in_pad = ip;
    maxw = std::max({maxw, ip, H});
    flops += 2.0 * G * H * ((double)m.gru.I + H);
    wbytes += 4.0 * ((double)G * H * (m.gru.I + H) + 2.0 * G * H);
    const size_t sw = (size_t)p.gru.sw;
    e.d_hidden = e.dalloc<float>((size_t)e.opts.max_batch * sw);
    hip_check(hipMemsetAsync(e.d_hidden, 0, (size_t)e.opts.max_batch * sw * sizeof(float), e.stream), "hipMemsetAsync");
  } else {
    p.in_pad = p.L[0].K_pad;
  }
  p.lds_stride = maxw + 4;  // +16 B per row: rows start on different LDS banks
  // Every LDS column a layer reads is written first (hidden N_pad == next K_pad,
  // the observation stage writes [0, in_pad)), except after a GRU whose H is not
  // a multiple of 64: then the columns [H, ceil64(H)) must be cleared once.
  p.zero_fill = (m.has_gru && m.gru.H % 64) ? 1 : 0;
  // head fusion: a narrow final layer (<= 2 tiles) whose predecessor runs one tile
  // group set per wave (T >= waves) is folded into the predecessor's epilogue
  if (p.nl >= 2 && !std::getenv("GO2PI_NO_HEAD_FUSE")) {  // env: A/B diagnostics only
    const int t_last = p.L[p.nl - 1].N_pad / 16, t_prev = p.L[p.nl - 2].N_pad / 16;
    if (t_last <= 2 && t_prev >= e.waves) p.head_fuse = t_last;
  }
  // 4-wave uniform-MLP pipeline (kernels.hip, w4_step): a fused head, and
  // every hidden layer exactly one group of 2, 4 or 8 tiles per wave. It is the
  // default (waves = 0) wherever it applies: measured faster than the generic
  // 8-wave body; otherwise waves = 0 means 8.
  // (a GRU policy runs its cell first and hands h' to the pipeline as layer 0's input)
  if (w4_shape) {
    const int t_last = p.L[p.nl - 1].N_pad / 16;
    const int tpw = p.L[0].N_pad / 64;
    {
      e.waves = 4;
      p.head_fuse = t_last;
      p.w4_tpw = tpw;
      p.w4_bias = (p.nl - 1) * 64 * tpw;
      std::vector<float> pack(p.w4_bias);
      for (int l = 0; l + 1 < p.nl; ++l)
        hip_check(hipMemcpy(pack.data() + (size_t)l * 64 * tpw, p.L[l].bias, sizeof(float) * 64 * tpw,
                            hipMemcpyDeviceToHost),
                  "hipMemcpy");
      p.w4_bpack = e.upload(pack);
    }
  }

  // prologue: model-defined (Sub/Div/Mul/Clip nodes) and/or opts-defined normalisation
  std::vector<float> sub = m.pre_sub, div = m.pre_div;
  if (e.opts.obs_mean) {
    if (!sub.empty()) throw ApiError("model already normalises its input; obs_mean not allowed", GO2PI_E_INVALID);
    sub.assign(e.opts.obs_mean, e.opts.obs_mean + m.in_dim);
  }
  if (e.opts.obs_std) {
    if (!div.empty()) throw ApiError("model already normalises its input; obs_std not allowed", GO2PI_E_INVALID);
    div.assign(e.opts.obs_std, e.opts.obs_std + m.in_dim);
  }
  if (!sub.empty()) { p.pre_sub = e.upload(sub); p.pre_sub_bcast = sub.size() == 1; }
  if (!div.empty()) { p.pre_div = e.upload(div); p.pre_div_bcast = div.size() == 1; }
  if (!m.pre_mul.empty()) {
    if (e.opts.obs_mean || e.opts.obs_std)
      throw ApiError("model already scales its input; obs_mean / obs_std not allowed", GO2PI_E_INVALID);
    p.pre_mul = e.upload(m.pre_mul);
    p.pre_mul_bcast = m.pre_mul.size() == 1;
  }
  p.obs_lo = m.pre_lo;
  p.obs_hi = m.pre_hi;
  if (e.opts.obs_clip > 0.f) {
    p.obs_lo = std::max(p.obs_lo, -e.opts.obs_clip);
    p.obs_hi = std::min(p.obs_hi, e.opts.obs_clip);
  }
  p.pre_clip = (std::isfinite(p.obs_lo) || std::isfinite(p.obs_hi)) ? 1 : 0;
  // action epilogue: the graph's trailing Clip / scalar Mul (post_fn: clip, then
  // scale), then the options'. The options apply after the graph, which post_fn's
  // fixed order tanh -> clip -> scale can only express when the graph adds no scale
  // (and, for tanh, no clip either).
  const bool m_clip = std::isfinite(m.clip_lo) || std::isfinite(m.clip_hi);
  if (e.opts.action_tanh && (m_clip || m.post_scale != 1.f))
    throw ApiError("action_tanh on a graph that clips or scales its output is not supported", GO2PI_E_INVALID);
  if (e.opts.action_clip > 0.f && m.post_scale != 1.f)
    throw ApiError("action_clip on a graph that scales its output is not supported", GO2PI_E_INVALID);
  p.post_tanh = e.opts.action_tanh ? 1 : 0;
  p.clip_lo = m.clip_lo;
  p.clip_hi = m.clip_hi;
  if (e.opts.action_clip > 0.f) {
    p.clip_lo = std::max(p.clip_lo, -e.opts.action_clip);
    p.clip_hi = std::min(p.clip_hi, e.opts.action_clip);
  }
  p.scale = m.post_scale * ((e.opts.action_scale != 0.f) ? e.opts.action_scale : 1.f);

  const size_t lds = go2pi::fused_lds_bytes(p, e.waves);
  if (lds > 160 * 1024)
    throw ApiError("layer width " + std::to_string(maxw) + " needs " + std::to_string(lds) +
                   " B of LDS per tile (> 160 KiB)", GO2PI_E_MODEL);

  // buffers
  e.d_obs = e.dalloc<float>((size_t)e.opts.max_batch * m.in_dim);
  e.d_act = e.dalloc<float>((size_t)e.opts.max_batch * m.out_dim);
  e.tmp_stride = maxw;
  e.d_tmp[0] = e.dalloc<float>((size_t)GO2PI_SMALL_MAXB * maxw);
  e.d_tmp[1] = e.dalloc<float>((size_t)GO2PI_SMALL_MAXB * maxw);
  e.palloc(&e.h_obs, &e.m_obs, sizeof(float) * GO2PI_SMALL_MAXB * m.in_dim);
  e.palloc(&e.h_act, &e.m_act, sizeof(float) * GO2PI_SMALL_MAXB * m.out_dim);

  // single-launch small-batch path: dense programs whose layers fit the kernel's
  // register slots (K_pad <= 1024) and whose widest layer fits one resident grid
  {
    int kmax = 0;
    for (int l = 0; l < p.nl; ++l) kmax = std::max(kmax, p.L[l].K_pad);
    const bool lat_shape = kmax <= 1024 && go2pi::latency_grid(p) <= 256 && e.small_batch > 0 &&
                           !std::getenv("GO2PI_SMALL_CHAIN");  // env: diagnostics, force the GEMV chain
    e.latency_ok = !m.has_gru && lat_shape;
    // the resident kernel's GRU / LSTM form (resident.hip, RNN): the cell tiled in front
    // of the dense layers, h' carried between requests as granules (an LSTM's c in the
    // owning workgroups' LDS)
    const bool res_rnn = m.has_gru && ((m.gru.cell == 0 && m.gru.lbr == 1) || m.gru.cell == 1) && m.gru.H % 64 == 0 &&
                         p.gru.I_pad + m.gru.H <= 512 && (m.gru.H >> 4) <= 256 && lat_shape && e.opts.resident_ms > 0;
    e.palloc(&e.h_err, &e.m_err, 512);
    p.err = e.m_err + 64;  // batched kernel hand-off timeouts
    if (e.latency_ok || res_rnn) {
      e.gstride = GO2PI_SMALL_MAXB * maxw;
      const size_t ng = (size_t)std::max(1, p.nl - 1) * e.gstride;
      e.d_gran = e.dalloc<unsigned long long>(ng);
      hip_check(hipMemsetAsync(e.d_gran, 0, ng * sizeof(unsigned long long), e.stream), "hipMemsetAsync");
      e.h_done = e.h_err + 32;  // 128 B apart: its own cache line
      e.m_done = e.m_err + 32;
      e.done_ok = p.L[p.nl - 1].N_pad == 16;
    }
    if (res_rnn && e.done_ok) e.d_hgran = e.dalloc<unsigned long long>(2 * (size_t)GO2PI_SMALL_MAXB * m.gru.H);
    // resident path: the latency kernel's program shape, the request ring in host memory
    if ((e.latency_ok || res_rnn) && e.done_ok && e.opts.resident_ms > 0) {
      // room for a controller tick's rows too (GO2PI_CTL_RAW + in_dim floats per robot)
      const size_t nreq = 1 + GO2PI_SMALL_MAXB * (size_t)(m.in_dim + GO2PI_CTL_RAW);
      size_t rb = sizeof(unsigned long long) * nreq;
      if (void *bar = bar_take(e.device, rb)) {  // large BAR: the ring in VRAM, written by the host
        e.h_req = e.m_req = static_cast<unsigned long long *>(bar);
        e.req_bar_bytes = rb;
      } else {
        e.palloc(&e.h_req, &e.m_req, sizeof(unsigned long long) * nreq);
      }
      // (the controller form's answer granules too: ctl_gran)
      e.n_actg = std::max((size_t)GO2PI_SMALL_MAXB * m.out_dim, (size_t)go2pi::ctl_gran(m.in_dim).total);
      e.palloc(&e.h_actg, &e.m_actg, sizeof(unsigned long long) * e.n_actg);
      e.d_mirror = e.dalloc<unsigned long long>(1 + GO2PI_SMALL_MAXB * (size_t)m.in_dim);
      int khz = 0;
      hip_check(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, e.device), "hipDeviceGetAttribute");
      if (khz <= 0) khz = 100000;
      e.res_idle_ticks = (unsigned long long)e.opts.resident_ms * (unsigned long long)khz;
      e.resident_ok = true;
      res_register(&e);
      e.resident_ctl_ok = !m.has_gru;  // the controller-tick form serves dense policies
    }
  }
  if (std::getenv("GO2PI_DIAG_STAMPS")) {  // diagnostics: per-workgroup clock stamps
    e.n_stamps = GO2PI_STAMPS_PER_WG * ((e.opts.max_batch + GO2PI_TILE_ROWS - 1) / GO2PI_TILE_ROWS);
    p.stamps = e.dalloc<unsigned long long>(e.n_stamps);
    hip_check(hipMemsetAsync(p.stamps, 0, e.n_stamps * sizeof(unsigned long long), e.stream), "hipMemsetAsync");
  }
  // the finished program, copied to device memory for the latency kernel
  {
    float *z = e.dalloc<float>(64);
    hip_check(hipMemsetAsync(z, 0, 64 * sizeof(float), e.stream), "hipMemsetAsync");
    p.zero = z;
  }
  // controller tick: a policy with kHistory x 49 observations and 12 actions
  if (m.in_dim > 0 && m.in_dim % GO2PI_CTL_STEP_DIM == 0 && m.in_dim <= 16 * GO2PI_CTL_STEP_DIM &&
      m.out_dim == GO2PI_CTL_DOF) {
    e.ctl_hist = m.in_dim / GO2PI_CTL_STEP_DIM;
    e.d_ctl = e.dalloc<go2pi::DevCtlParams>(1);
    go2pi_ctl_params cp;
    go2pi_ctl_default_params(&cp);
    set_ctl_params(e, cp);
  }
  p.yield = yield_word(e.device);
  // the pipeline's hot block (program.hpp): what it reads, in one scalar burst
  if (p.w4_tpw) {
    const auto &H = p.L[p.nl - 1];
    p.l0_w = p.L[0].w;
    p.head_w = H.w;
    p.head_bias = H.bias;
    p.bpack = p.w4_bpack;
    p.zero_hot = p.zero;
    p.err_hot = p.err;
    p.nbias = p.w4_bias;
    p.head_n = H.N;
    p.c0 = p.L[0].K_pad / 16;
    p.in_dim_hot = p.in_dim;
    p.hid_act = p.L[0].act;
    p.hid_alpha = p.L[0].alpha;
    p.hid_beta = p.L[0].beta;
    p.head_act = H.act;
    p.head_alpha = H.alpha;
    p.head_beta = H.beta;
    p.post_plain = (!p.post_tanh && std::isinf(p.clip_lo) && p.clip_lo < 0 && std::isinf(p.clip_hi) &&
                    p.clip_hi > 0 && p.scale == 1.f) ? 1 : 0;
    p.w4_c0m = p.c0 % 4;
    // the lean kernel: no prologue / epilogue arithmetic, no recurrent cell, and an
    // LDS row no wider than the hidden layers
    p.w4_plain = !p.has_gru && !p.pre_sub && !p.pre_div && !p.pre_mul && !p.pre_clip && !p.post_tanh &&
                 std::isinf(p.clip_lo) && p.clip_lo < 0 && std::isinf(p.clip_hi) && p.clip_hi > 0 &&
                 p.scale == 1.f && p.lds_stride == 64 * p.w4_tpw + 4 && !std::getenv("GO2PI_NO_PLAIN");
    // the lean kernel's compile-time activation: Elu (the exported rsl_rl / Isaac policies'), else runtime
    // (1 = Elu with alpha 1, the ONNX default; any other alpha takes the runtime form)
    p.w4_actc = (p.hid_act == 1 && p.hid_alpha == 1.f && !std::getenv("GO2PI_LEAN_RT_ACT")) ? 1 : -1;  // env: A/B only
    // ... and its hidden-layer count (3: the usual policy depth): the layer loop fully
    // unrolled, so no ring-register copies (and no vmcnt(0)) at the layer boundaries.
    // The general body (recurrent policies) takes both only together.
    p.w4_nhc = (p.w4_actc == 1 && p.nl - 1 == 3 && !std::getenv("GO2PI_LEAN_RT_NH")) ? 3 : 0;  // env: A/B only
    if (!p.w4_plain && p.w4_nhc == 0) p.w4_actc = -1;
    // the lean recurrent tick (policy_gru_kernel, r05; policy_lstm_kernel, r06): a GRU cell
    // (lbr = 1) or an LSTM cell in front of a dense chain the lean kernel would serve
    // (gru_lean_on: GO2PI_GRU_GENERAL=1 keeps the general body for both cells, A/B)
    p.w4_gru_lean = (p.has_gru && ((p.gru.cell == 0 && p.gru.lbr == 1) || p.gru.cell == 1) &&
                     (p.gru.H == 128 || p.gru.H == 256) &&
                     p.gru.H <= 64 * p.w4_tpw && !p.pre_sub && !p.pre_div && !p.pre_mul && !p.pre_clip &&
                     p.post_plain && p.lds_stride == 64 * p.w4_tpw + 4 && p.w4_actc == 1 && p.w4_nhc == 3 &&
                     p.c0 == p.gru.H / 16 && p.gru.I_pad == (p.in_dim + 63) / 64 * 64 && p.in_dim < 4096 &&
                     !p.zero_fill && gru_lean_on()) ? 1 : 0;
  }
  // a dense policy whose weights fit one CU's registers is served by the single-
  // workgroup resident kernel (no inter-workgroup hop per layer; GO2PI_RES_MULTI=1:
  // the multi-workgroup form, A/B diagnostics)
  e.resident1 = e.resident_ok && !m.has_gru && go2pi::resident1_fits(p, false) && !std::getenv("GO2PI_RES_MULTI");
  e.resident1_ctl = e.resident_ok && !m.has_gru && go2pi::resident1_fits(p, true) && !std::getenv("GO2PI_RES_MULTI");
  e.ctl_gran_ok = e.resident1_ctl && go2pi::resident1_ctl_granules(p);
  // the controller tick's general body instead of the lean tick kernel (A/B diagnostics,
  // tests/test_gpu_controller.py::test_controller_tick_bodies)
  p.ctl_general = std::getenv("GO2PI_CTL_GENERAL") != nullptr ? 1 : 0;
  // a wide dense policy (every hidden layer 256 or 512 wide: BASELINE configs[1]'s
  // 48 -> 512^3 -> 12) is served by policy_wide_kernel when every workgroup can poll the
  // request ring in device memory (large BAR); else by the multi-workgroup kernel, whose
  // workgroup 0 alone polls the host and mirrors the request (GO2PI_RES_MULTI=1: that
  // form regardless, A/B and its tests)
  e.wide = e.resident_ok && !e.resident1 && !m.has_gru && e.req_bar_bytes > 0 && go2pi::wide_shape(p).nl > 0 &&
           !std::getenv("GO2PI_RES_MULTI");
  hip_check(go2pi::configure_kernels(p, e.waves), "hipFuncSetAttribute");
  e.d_prog = e.dalloc<go2pi::DevProgram>(1);
  hip_check(hipMemcpy(e.d_prog, &p, sizeof(p), hipMemcpyHostToDevice), "hipMemcpy");
  // (not hipDeviceSynchronize: that would wait for other engines' resident kernels)
  hip_check(hipStreamSynchronize(e.stream), "hipStreamSynchronize");
  hip_check(hipStreamSynchronize(nullptr), "hipStreamSynchronize");

  e.cost.flops_per_row = flops;
  e.cost.weight_bytes = wbytes;
  e.cost.io_bytes_per_row = 4.0 * (m.in_dim + m.out_dim) + (m.has_gru ? 8.0 * p.gru.sw : 0.0);
  e.cost.n_layers = p.nl;
  e.cost.has_gru = p.has_gru ? (p.gru.cell == 1 ? 2 : 1) : 0;  // 1 GRU, 2 LSTM (go2pi.h)
}

// Every C-ABI entry point runs through here: exceptions become status codes, and
// the caller's current HIP device is restored on the way out.
// (no DeviceRestore: go2pi_run's resident fast path, which switches devices lazily)
template <class F>
int guarded_nodev(F &&f) {
  try {
    g_last_error.clear();
    return f();
  } catch (const ApiError &ex) {
    g_last_error = ex.what();
    return ex.code;
  } catch (const HipError &ex) {
    g_last_error = ex.what();
    return ex.code;
  } catch (const std::exception &ex) {
    g_last_error = ex.what();
    return GO2PI_E_INVALID;
  }
}

template <class F>
int guarded(F &&f) {
  DeviceRestore keep;
  try {
    g_last_error.clear();
    return f();
  } catch (const ApiError &ex) {
    g_last_error = ex.what();
    return ex.code;
  } catch (const HipError &ex) {
    g_last_error = ex.what();
    return ex.code;
  } catch (const std::bad_alloc &) {
    g_last_error = "out of host memory";
    return GO2PI_E_INVALID;
  } catch (const std::exception &ex) {
    g_last_error = ex.what();
    return GO2PI_E_INVALID;
  }
}

void check_engine(const go2pi_engine *e) {
  if (!e) throw ApiError("null engine", GO2PI_E_INVALID);
}
// Mutating calls: the resident kernel (if any) leaves first, so the stream is free.
void check_engine(go2pi_engine *e) {
  if (!e) throw ApiError("null engine", GO2PI_E_INVALID);
  (void)hipSetDevice(e->device);
  e->resident_stop();
}

void check_batch(const go2pi_engine *e, int64_t batch) {
  if (batch < 0) throw ApiError("negative batch", GO2PI_E_INVALID);
  if (batch > e->opts.max_batch)
    throw ApiError("batch " + std::to_string(batch) + " exceeds max_batch " + std::to_string(e->opts.max_batch),
                   GO2PI_E_CAPACITY);
}

}  // namespace

extern "C" {

void go2pi_default_opts(go2pi_opts *o) {
  if (!o) return;
  std::memset(o, 0, sizeof(*o));
  o->struct_size = sizeof(go2pi_opts);
  o->device = 0;
  o->max_batch = 4096;
  o->use_graph = 1;
  o->log_level = 2;
  o->waves = 0;
  o->small_batch = 0;
  o->obs_clip = 0.f;
  o->action_tanh = 0;
  o->action_clip = 0.f;
  o->action_scale = 0.f;
}

int go2pi_create_from_memory(const void *bytes, size_t nbytes, const go2pi_opts *opts, go2pi_engine **out) {
  return guarded([&] {
    if (!out) throw ApiError("null output pointer", GO2PI_E_INVALID);
    *out = nullptr;
    if (!bytes || !nbytes) throw ApiError("empty model buffer", GO2PI_E_MODEL);
    auto e = std::make_unique<go2pi_engine>();
    build(*e, static_cast<const uint8_t *>(bytes), nbytes, opts);
    *out = e.release();
    return GO2PI_OK;
  });
}

int go2pi_create(const char *path, const go2pi_opts *opts, go2pi_engine **out) {
  return guarded([&] {
    if (!out) throw ApiError("null output pointer", GO2PI_E_INVALID);
    *out = nullptr;
    if (!path) throw ApiError("null model path", GO2PI_E_INVALID);
    std::ifstream f(path, std::ios::binary);
    if (!f) throw ApiError(std::string("cannot open model file '") + path + "'", GO2PI_E_MODEL);
    std::vector<uint8_t> buf((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
    if (buf.empty()) throw ApiError(std::string("empty model file '") + path + "'", GO2PI_E_MODEL);
    auto e = std::make_unique<go2pi_engine>();
    build(*e, buf.data(), buf.size(), opts);
    *out = e.release();
    return GO2PI_OK;
  });
}

void go2pi_destroy(go2pi_engine *e) { delete e; }

int go2pi_num_io(const go2pi_engine *e, int32_t *ni, int32_t *no) {
  return guarded([&] {
    check_engine(e);
    if (ni) *ni = (int32_t)e->model.inputs.size();
    if (no) *no = (int32_t)e->model.outputs.size();
    return GO2PI_OK;
  });
}

int go2pi_io_name(const go2pi_engine *e, int32_t is_output, int32_t index, char *buf, size_t cap) {
  return guarded([&] {
    check_engine(e);
    const auto &v = is_output ? e->model.outputs : e->model.inputs;
    if (index < 0 || index >= (int32_t)v.size()) throw ApiError("io index out of range", GO2PI_E_INVALID);
    if (!buf || cap == 0) throw ApiError("null name buffer", GO2PI_E_INVALID);
    const std::string &s = v[index].name;
    const size_t k = std::min(cap - 1, s.size());
    std::memcpy(buf, s.data(), k);
    buf[k] = 0;
    return GO2PI_OK;
  });
}

int go2pi_io_shape(const go2pi_engine *e, int32_t is_output, int32_t index, int64_t *dims, int32_t cap,
                   int32_t *rank) {
  return guarded([&] {
    check_engine(e);
    const auto &v = is_output ? e->model.outputs : e->model.inputs;
    if (index < 0 || index >= (int32_t)v.size()) throw ApiError("io index out of range", GO2PI_E_INVALID);
    const auto &s = v[index].shape;
    if (rank) *rank = (int32_t)s.size();
    for (int32_t i = 0; dims && i < cap && i < (int32_t)s.size(); ++i) dims[i] = s[i];
    return GO2PI_OK;
  });
}

int go2pi_io_dims(const go2pi_engine *e, int64_t *in_dim, int64_t *out_dim) {
  return guarded([&] {
    check_engine(e);
    if (in_dim) *in_dim = e->model.in_dim;
    if (out_dim) *out_dim = e->model.out_dim;
    return GO2PI_OK;
  });
}

int go2pi_run(go2pi_engine *e, const float *obs, float *act, int64_t batch) {
  // batch <= 8 on a live resident kernel: served with no HIP runtime call (the device
  // switch and its restore were three HIP API entries per act(), on the 5 us path).
  // Invariant: this skips check_engine / check_batch because a live kernel
  // (resident_ready: resident_live) exists only after an earlier call on this engine
  // passed them in the guarded path below (resident_start is reached from there only),
  // and the fields read here (opts, resident_ok, model dims) never change after build.
  // The batch bounds are re-checked in the condition itself.
  bool res_try = true;
  if (e && obs && act && batch >= 1 && batch <= GO2PI_SMALL_MAXB && batch <= e->opts.max_batch && e->resident_ok &&
      e->resident_ready(nullptr)) {
    e->lazy_dev = true;
    const int rc = guarded_nodev([&] {
      const bool ok = e->resident_serve(nullptr, obs, batch, 0u);
      if (ok) {
        e->check_handoff();
        std::memcpy(act, e->h_act, sizeof(float) * (size_t)batch * e->model.out_dim);
      }
      return ok ? GO2PI_OK : 1;
    });
    e->dev_done();
    if (rc != 1) return rc;
    res_try = false;  // not served (evicted twice): a launch serves it
  }
  return guarded([&] {
    check_engine(static_cast<const go2pi_engine *>(e));
    check_batch(e, batch);
    if (batch == 0) return GO2PI_OK;
    if (!obs || !act) throw ApiError("null obs/act buffer", GO2PI_E_INVALID);
    hip_check(hipSetDevice(e->device), "hipSetDevice");
    if (res_try && e->resident_ok && batch <= GO2PI_SMALL_MAXB && e->resident_serve(nullptr, obs, batch, 0u)) {
      e->check_handoff();
      std::memcpy(act, e->h_act, sizeof(float) * (size_t)batch * e->model.out_dim);
      return GO2PI_OK;
    }
    e->resident_stop();
    std::unique_lock<std::mutex> ev;  // (held until the launch below is enqueued)
    if (batch > GO2PI_SMALL_MAXB || !e->latency_ok) ev = evict_residents(e, batch);  // a batched (fused) launch follows
    const size_t in_b = sizeof(float) * (size_t)batch * e->model.in_dim;
    const size_t out_b = sizeof(float) * (size_t)batch * e->model.out_dim;
    if (batch <= GO2PI_SMALL_MAXB) {
      // pinned host-mapped staging: kernels read obs / write act over PCIe directly
      std::memcpy(e->h_obs, obs, in_b);
      bool synced = false;
      if (e->use_latency(batch)) {
        // one direct launch (per-call epoch argument); completion observed by spinning on
        // the host-mapped done word (a stream sync costs ~10 us more on this stack)
        e->enqueue(e->m_obs, e->m_act, batch, e->stream, e->done_ok ? e->m_done : nullptr);
        if (e->done_ok) synced = e->spin_done();
      } else if (!e->opts.use_graph) {
        e->enqueue(e->m_obs, e->m_act, batch, e->stream);
      } else {
        hip_check(hipGraphLaunch(e->graph_for((int)batch), e->stream), "hipGraphLaunch");
      }
      if (ev.owns_lock()) ev.unlock();  // (the launch is enqueued)
      if (!synced) hip_check(hipStreamSynchronize(e->stream), "hipStreamSynchronize");
      e->check_handoff();
      std::memcpy(act, e->h_act, out_b);
    } else {
      hip_check(hipMemcpyAsync(e->d_obs, obs, in_b, hipMemcpyHostToDevice, e->stream), "hipMemcpyAsync H2D");
      e->enqueue(e->d_obs, e->d_act, batch, e->stream);
      if (ev.owns_lock()) ev.unlock();  // (the launch is enqueued)
      hip_check(hipMemcpyAsync(act, e->d_act, out_b, hipMemcpyDeviceToHost, e->stream), "hipMemcpyAsync D2H");
      hip_check(hipStreamSynchronize(e->stream), "hipStreamSynchronize");
      e->check_handoff();
    }
    return GO2PI_OK;
  });
}

int go2pi_run_device(go2pi_engine *e, const float *obs_dev, float *act_dev, int64_t batch, void *hip_stream) {
  return guarded([&] {
    check_engine(e);
    check_batch(e, batch);
    if (batch == 0) return GO2PI_OK;
    if (!obs_dev || !act_dev) throw ApiError("null obs/act buffer", GO2PI_E_INVALID);
    hip_check(hipSetDevice(e->device), "hipSetDevice");
    e->check_handoff();  // a failure of an earlier asynchronous launch surfaces here (or at go2pi_sync)
    std::unique_lock<std::mutex> ev;  // (held until the launch is enqueued)
    if (!e->use_latency(batch)) ev = evict_residents(e, batch);
    e->enqueue(obs_dev, act_dev, batch, static_cast<hipStream_t>(hip_stream));
    return GO2PI_OK;
  });
}

int go2pi_run_sequence_device(go2pi_engine *e, const float *obs_dev, float *act_dev, int64_t steps, int64_t batch,
                              void *hip_stream) {
  return guarded([&] {
    check_engine(e);
    check_batch(e, batch);
    if (steps < 0) throw ApiError("negative steps", GO2PI_E_INVALID);
    if (batch == 0 || steps == 0) return GO2PI_OK;
    if (!obs_dev || !act_dev) throw ApiError("null obs/act buffer", GO2PI_E_INVALID);
    if ((double)steps * batch * std::max(e->model.in_dim, e->model.out_dim) > 2147483647.0 * 4)
      throw ApiError("sequence too large", GO2PI_E_INVALID);
    hip_check(hipSetDevice(e->device), "hipSetDevice");
    hipStream_t s = static_cast<hipStream_t>(hip_stream);
    const auto ev = evict_residents(e, batch);  // (held until the launch is enqueued)
    hip_check(go2pi::launch_policy_fused(e->prog, e->d_prog, e->waves, obs_dev, act_dev, e->d_hidden, (int)batch,
                                         (int)steps, s),
              "fused sequence launch");
    return GO2PI_OK;
  });
}

int go2pi_hidden_dim(const go2pi_engine *e, int64_t *hd) {
  return guarded([&] {
    check_engine(e);
    if (hd) *hd = e->model.has_gru ? e->prog.gru.sw : 0;  // LSTM: h | c
    return GO2PI_OK;
  });
}

int go2pi_reset_hidden(go2pi_engine *e, const uint8_t *mask, int64_t batch) {
  return guarded([&] {
    check_engine(e);
    if (!e->model.has_gru) return GO2PI_OK;
    hip_check(hipSetDevice(e->device), "hipSetDevice");
    const int H = e->prog.gru.sw;  // state floats per robot
    if (!mask) {
      hip_check(hipMemsetAsync(e->d_hidden, 0, sizeof(float) * (size_t)e->opts.max_batch * H, e->stream), "hipMemsetAsync");
    } else {
      check_batch(e, batch);
      // coalesce runs of reset rows into single memsets
      int64_t i = 0;
      while (i < batch) {
        if (!mask[i]) { ++i; continue; }
        int64_t j = i;
        while (j < batch && mask[j]) ++j;
        hip_check(hipMemsetAsync(e->d_hidden + (size_t)i * H, 0, sizeof(float) * (size_t)(j - i) * H, e->stream),
                  "hipMemsetAsync");
        i = j;
      }
    }
    hip_check(hipStreamSynchronize(e->stream), "hipStreamSynchronize");
    return GO2PI_OK;
  });
}

int go2pi_get_hidden(go2pi_engine *e, float *h, int64_t batch) {
  return guarded([&] {
    check_engine(e);
    check_batch(e, batch);
    if (!e->model.has_gru || batch == 0) return GO2PI_OK;
    if (!h) throw ApiError("null hidden buffer", GO2PI_E_INVALID);
    hip_check(hipSetDevice(e->device), "hipSetDevice");
    hip_check(hipStreamSynchronize(e->stream), "hipStreamSynchronize");
    hip_check(hipMemcpy(h, e->d_hidden, sizeof(float) * (size_t)batch * e->prog.gru.sw, hipMemcpyDeviceToHost),
              "hipMemcpy D2H");
    return GO2PI_OK;
  });
}

int go2pi_set_hidden(go2pi_engine *e, const float *h, int64_t batch) {
  return guarded([&] {
    check_engine(e);
    check_batch(e, batch);
    if (!e->model.has_gru || batch == 0) return GO2PI_OK;
    if (!h) throw ApiError("null hidden buffer", GO2PI_E_INVALID);
    hip_check(hipSetDevice(e->device), "hipSetDevice");
    hip_check(hipStreamSynchronize(e->stream), "hipStreamSynchronize");
    hip_check(hipMemcpy(e->d_hidden, h, sizeof(float) * (size_t)batch * e->prog.gru.sw, hipMemcpyHostToDevice),
              "hipMemcpy H2D");
    return GO2PI_OK;
  });
}

void go2pi_ctl_default_params(go2pi_ctl_params *p) {
  if (!p) return;
  std::memset(p, 0, sizeof(*p));
  p->struct_size = sizeof(go2pi_ctl_params);
  p->kp = 28.f;  // controller.hpp:119-120
  p->kd = 0.5f;
  p->kp_stop = 5.f;           // controller.cpp:246
  p->action_limit = 1000.f;   // kActionLimit, controller.hpp:17
  p->contact_threshold = 22.f;  // controller.hpp:100-103
  p->gravity_w[2] = -1.f;     // gravity_w_, controller.hpp:131
  p->action_scale = 0.25;     // controller.cpp:244
  static const double q0[12] = {0.1, -0.1, 0.1, -0.1, 0.8, 0.8, 1.0, 1.0, -1.5, -1.5, -1.5, -1.5};  // controller.hpp:165
  std::memcpy(p->q0, q0, sizeof(q0));
}

int go2pi_ctl_history(const go2pi_engine *e, int32_t *hist) {
  return guarded([&] {
    check_engine(e);
    if (!e->ctl_hist)
      throw ApiError("policy I/O is not a Go2 controller's (obs " + std::to_string(e->model.in_dim) +
                         " not a multiple of 49, or action " + std::to_string(e->model.out_dim) + " != 12)",
                     GO2PI_E_MODEL);
    if (hist) *hist = e->ctl_hist;
    return GO2PI_OK;
  });
}

int go2pi_ctl_set_params(go2pi_engine *e, const go2pi_ctl_params *p) {
  return guarded([&] {
    check_engine(e);
    if (!p) throw ApiError("null params", GO2PI_E_INVALID);
    if (p->struct_size != (int32_t)sizeof(go2pi_ctl_params))
      throw ApiError("go2pi_ctl_params.struct_size mismatch", GO2PI_E_INVALID);
    if (!e->ctl_hist) throw ApiError("policy I/O is not a Go2 controller's", GO2PI_E_MODEL);
    hip_check(hipSetDevice(e->device), "hipSetDevice");
    hip_check(hipStreamSynchronize(e->stream), "hipStreamSynchronize");
    set_ctl_params(*e, *p);
    return GO2PI_OK;
  });
}

namespace {
// byte offsets of the controller staging buffers for `rows` robots (256 B aligned)
struct CtlLayout {
  size_t state, joy, obs, action, q_des, kp, kd, status, total;
  CtlLayout(int64_t rows, int in_dim) {
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    size_t o = 0;
    state = o; o = al(o + sizeof(float) * rows * GO2PI_CTL_STATE_DIM);
    joy = o; o = al(o + sizeof(float) * rows * GO2PI_CTL_JOY_DIM);
    obs = o; o = al(o + sizeof(float) * rows * in_dim);
    action = o; o = al(o + sizeof(float) * rows * GO2PI_CTL_DOF);
    q_des = o; o = al(o + sizeof(double) * rows * GO2PI_CTL_DOF);
    kp = o; o = al(o + sizeof(double) * rows * GO2PI_CTL_DOF);
    kd = o; o = al(o + sizeof(double) * rows * GO2PI_CTL_DOF);
    status = o; o = al(o + sizeof(uint32_t) * rows);
    total = o;
  }
};

void check_ctl(const go2pi_engine *e, int64_t batch) {
  check_engine(e);
  check_batch(e, batch);
  if (!e->ctl_hist) throw ApiError("policy I/O is not a Go2 controller's (need 49*k obs, 12 actions)", GO2PI_E_MODEL);
}
}  // namespace

int go2pi_controller_step(go2pi_engine *e, const float *state, const float *joy, float *obs, float *action,
                          double *q_des, double *kp, double *kd, uint32_t *status, int64_t batch) {
  // batch <= 8 on a live controller-form resident kernel: no HIP runtime call and no
  // input staging (the rows travel in the request itself; go2pi_run's fast path).
  // Invariant: check_ctl is skipped; the condition itself requires ctl_hist
  // (a controller policy: check_ctl's model test), the batch bounds and the staging
  // (h_ctl), and resident_ready(&all) requires a live controller-form kernel, which only
  // the guarded path below starts.
  bool res_try = true;
  if (e && state && obs && action && batch >= 1 && batch <= GO2PI_SMALL_MAXB && batch <= e->opts.max_batch &&
      e->ctl_hist && e->resident_ok && e->resident_ctl_ok && e->done_ok && e->h_ctl) {
    const int in_dim = e->model.in_dim;
    const CtlLayout L(GO2PI_SMALL_MAXB, in_dim);
    go2pi::DevCtl all{};
    all.prm = e->d_ctl;
    char *dev = e->m_ctl;
    all.state = reinterpret_cast<const float *>(dev + L.state);
    all.joy = reinterpret_cast<const float *>(dev + L.joy);
    all.obs = reinterpret_cast<float *>(dev + L.obs);
    all.action = reinterpret_cast<float *>(dev + L.action);
    all.q_des = reinterpret_cast<double *>(dev + L.q_des);
    all.kp = reinterpret_cast<double *>(dev + L.kp);
    all.kd = reinterpret_cast<double *>(dev + L.kd);
    all.status = reinterpret_cast<uint32_t *>(dev + L.status);
    if (e->resident_ready(&all)) {
      e->lazy_dev = true;
      const int rc = guarded_nodev([&] {
        const size_t n_state = sizeof(float) * batch * GO2PI_CTL_STATE_DIM, n_joy = sizeof(float) * batch * GO2PI_CTL_JOY_DIM;
        const size_t n_obs = sizeof(float) * batch * in_dim, n_act = sizeof(float) * batch * GO2PI_CTL_DOF;
        const size_t n_d = sizeof(double) * batch * GO2PI_CTL_DOF, n_st = sizeof(uint32_t) * batch;
        const unsigned flags = (joy ? GO2PI_RES_JOY : 0u) | (q_des ? GO2PI_RES_QDES : 0u) | (kp ? GO2PI_RES_KP : 0u) |
                               (kd ? GO2PI_RES_KD : 0u) | (status ? GO2PI_RES_STATUS : 0u);
        float *rows = e->res_rows.data();  // state | joystick | obs | action
        std::memcpy(rows, state, n_state);
        if (joy) std::memcpy(rows + batch * GO2PI_CTL_STATE_DIM, joy, n_joy);
        else std::memset(rows + batch * GO2PI_CTL_STATE_DIM, 0, n_joy);
        std::memcpy(rows + batch * (GO2PI_CTL_STATE_DIM + GO2PI_CTL_JOY_DIM), obs, n_obs);
        std::memcpy(rows + batch * (GO2PI_CTL_STATE_DIM + GO2PI_CTL_JOY_DIM + in_dim), action, n_act);
        if (!e->resident_serve(&all, rows, batch, flags)) return 1;
        e->check_handoff();
        if (e->ctl_gran_ok) {
          e->ctl_take(batch, obs, action, q_des, kp, kd, status);
          return GO2PI_OK;
        }
        std::memcpy(obs, e->h_ctl + L.obs, n_obs);
        std::memcpy(action, e->h_ctl + L.action, n_act);
        if (q_des) std::memcpy(q_des, e->h_ctl + L.q_des, n_d);
        if (kp) std::memcpy(kp, e->h_ctl + L.kp, n_d);
        if (kd) std::memcpy(kd, e->h_ctl + L.kd, n_d);
        if (status) std::memcpy(status, e->h_ctl + L.status, n_st);
        return GO2PI_OK;
      });
      e->dev_done();
      if (rc != 1) return rc;
      res_try = false;  // not served (evicted twice): a launch serves it
    }
  }
  return guarded([&] {
    check_ctl(e, batch);
    if (batch == 0) return GO2PI_OK;
    if (!state || !obs || !action) throw ApiError("null state/obs/action buffer", GO2PI_E_INVALID);
    hip_check(hipSetDevice(e->device), "hipSetDevice");
    const int in_dim = e->model.in_dim;
    const bool small = batch <= GO2PI_SMALL_MAXB;
    const CtlLayout L(small ? GO2PI_SMALL_MAXB : e->opts.max_batch, in_dim);
    const size_t n_state = sizeof(float) * batch * GO2PI_CTL_STATE_DIM, n_joy = sizeof(float) * batch * GO2PI_CTL_JOY_DIM;
    const size_t n_obs = sizeof(float) * batch * in_dim, n_act = sizeof(float) * batch * GO2PI_CTL_DOF;
    const size_t n_d = sizeof(double) * batch * GO2PI_CTL_DOF, n_st = sizeof(uint32_t) * batch;
    char *dev;  // device-side view of the staging
    if (small) {
      if (!e->h_ctl) {
        e->palloc(&e->h_ctl, &e->m_ctl, L.total);
      }
      std::memcpy(e->h_ctl + L.state, state, n_state);
      if (joy) std::memcpy(e->h_ctl + L.joy, joy, n_joy);
      std::memcpy(e->h_ctl + L.obs, obs, n_obs);
      std::memcpy(e->h_ctl + L.action, action, n_act);
      dev = e->m_ctl;
    } else {
      if (!e->d_ctlbuf) e->d_ctlbuf = e->dalloc<char>(L.total);
      dev = e->d_ctlbuf;
      auto h2d = [&](size_t off, const void *src, size_t n) {
        hip_check(hipMemcpyAsync(dev + off, src, n, hipMemcpyHostToDevice, e->stream), "hipMemcpyAsync H2D");
      };
      h2d(L.state, state, n_state);
      if (joy) h2d(L.joy, joy, n_joy);
      h2d(L.obs, obs, n_obs);
      h2d(L.action, action, n_act);
    }
    go2pi::DevCtl c{};
    c.prm = e->d_ctl;
    c.state = reinterpret_cast<const float *>(dev + L.state);
    c.joy = joy ? reinterpret_cast<const float *>(dev + L.joy) : nullptr;
    c.obs = reinterpret_cast<float *>(dev + L.obs);
    c.action = reinterpret_cast<float *>(dev + L.action);
    c.q_des = q_des ? reinterpret_cast<double *>(dev + L.q_des) : nullptr;
    c.kp = kp ? reinterpret_cast<double *>(dev + L.kp) : nullptr;
    c.kd = kd ? reinterpret_cast<double *>(dev + L.kd) : nullptr;
    c.status = status ? reinterpret_cast<uint32_t *>(dev + L.status) : nullptr;
    const bool res = res_try && small && e->resident_ok && e->resident_ctl_ok && e->done_ok;
    bool served = false;  // by the resident kernel
    if (res) {
      // the resident kernel's controller form: every optional row has its place in the
      // staging; the header's flags say which this call passed
      go2pi::DevCtl all = c;
      all.joy = reinterpret_cast<const float *>(dev + L.joy);
      all.q_des = reinterpret_cast<double *>(dev + L.q_des);
      all.kp = reinterpret_cast<double *>(dev + L.kp);
      all.kd = reinterpret_cast<double *>(dev + L.kd);
      all.status = reinterpret_cast<uint32_t *>(dev + L.status);
      const unsigned flags = (joy ? GO2PI_RES_JOY : 0u) | (q_des ? GO2PI_RES_QDES : 0u) | (kp ? GO2PI_RES_KP : 0u) |
                             (kd ? GO2PI_RES_KD : 0u) | (status ? GO2PI_RES_STATUS : 0u);
      float *rows = e->res_rows.data();  // state | joystick | obs | action
      std::memcpy(rows, state, n_state);
      if (joy) std::memcpy(rows + batch * GO2PI_CTL_STATE_DIM, joy, n_joy);
      else std::memset(rows + batch * GO2PI_CTL_STATE_DIM, 0, n_joy);
      std::memcpy(rows + batch * (GO2PI_CTL_STATE_DIM + GO2PI_CTL_JOY_DIM), obs, n_obs);
      std::memcpy(rows + batch * (GO2PI_CTL_STATE_DIM + GO2PI_CTL_JOY_DIM + in_dim), action, n_act);
      served = e->resident_serve(&all, rows, batch, flags);
    } else {
      e->resident_stop();
    }
    const bool single = !served && small && e->use_latency(batch) && e->done_ok;
    std::unique_lock<std::mutex> ev;
    if (!single && !served) ev = evict_residents(e, batch);  // a batched (fused) launch follows
    if (!served) e->enqueue_ctl(c, batch, e->stream, single ? e->m_done : nullptr);
    if (ev.owns_lock()) ev.unlock();  // (the launch is enqueued)
    if (small) {
      const bool synced = served || (single && e->spin_done());
      if (!synced) hip_check(hipStreamSynchronize(e->stream), "hipStreamSynchronize");
      e->check_handoff();
      if (served && e->ctl_gran_ok) {
        e->ctl_take(batch, obs, action, q_des, kp, kd, status);
      } else {
        std::memcpy(obs, e->h_ctl + L.obs, n_obs);
        std::memcpy(action, e->h_ctl + L.action, n_act);
        if (q_des) std::memcpy(q_des, e->h_ctl + L.q_des, n_d);
        if (kp) std::memcpy(kp, e->h_ctl + L.kp, n_d);
        if (kd) std::memcpy(kd, e->h_ctl + L.kd, n_d);
        if (status) std::memcpy(status, e->h_ctl + L.status, n_st);
      }
    } else {
      auto d2h = [&](void *dst, size_t off, size_t n) {
        hip_check(hipMemcpyAsync(dst, dev + off, n, hipMemcpyDeviceToHost, e->stream), "hipMemcpyAsync D2H");
      };
      d2h(obs, L.obs, n_obs);
      d2h(action, L.action, n_act);
      if (q_des) d2h(q_des, L.q_des, n_d);
      if (kp) d2h(kp, L.kp, n_d);
      if (kd) d2h(kd, L.kd, n_d);
      if (status) d2h(status, L.status, n_st);
      hip_check(hipStreamSynchronize(e->stream), "hipStreamSynchronize");
    }
    return GO2PI_OK;
  });
}

int go2pi_controller_step_device(go2pi_engine *e, const float *state, const float *joy, float *obs, float *action,
                                 double *q_des, double *kp, double *kd, uint32_t *status, int64_t batch,
                                 void *hip_stream) {
  return guarded([&] {
    check_ctl(e, batch);
    if (batch == 0) return GO2PI_OK;
    if (!state || !obs || !action) throw ApiError("null state/obs/action buffer", GO2PI_E_INVALID);
    hip_check(hipSetDevice(e->device), "hipSetDevice");
    // a live resident kernel shares the granules, epoch and error words the batch <= 8
    // launch uses: it leaves first (as for every other call on the engine)
    e->resident_stop();
    std::unique_lock<std::mutex> ev;  // (held until the launch is enqueued)
    if (!(e->use_latency(batch) && e->done_ok)) ev = evict_residents(e, batch);
    go2pi::DevCtl c{e->d_ctl, state, joy, obs, action, q_des, kp, kd, status};
    e->enqueue_ctl(c, batch, static_cast<hipStream_t>(hip_stream));
    return GO2PI_OK;
  });
}

int go2pi_sync(go2pi_engine *e) {
  return guarded([&] {
    check_engine(e);
    hip_check(hipSetDevice(e->device), "hipSetDevice");
    hip_check(hipStreamSynchronize(e->stream), "hipStreamSynchronize");
    e->check_handoff();
    return GO2PI_OK;
  });
}

int go2pi_get_cost(const go2pi_engine *e, go2pi_cost *c) {
  return guarded([&] {
    check_engine(e);
    if (!c) throw ApiError("null cost", GO2PI_E_INVALID);
    *c = e->cost;
    return GO2PI_OK;
  });
}

// the lean GRU tick wherever it applies (GO2PI_GRU_GENERAL=1: the general body, A/B;
// r05 same-box A/B, GRU-256 at 4096 robots: 56.7 against 60.5-60.9 us per one-tick launch)
static bool gru_lean_on() { return !std::getenv("GO2PI_GRU_GENERAL"); }

int go2pi_batched_kernel(const go2pi_engine *e, char *buf, size_t cap) {
  return guarded([&] {
    check_engine(e);
    if (!buf || cap == 0) throw ApiError("null buffer", GO2PI_E_INVALID);
    const int t = e->waves == 4 ? e->prog.w4_tpw : 0, h = t ? e->prog.head_fuse : 0;
    const int c0m = t ? e->prog.w4_c0m : 0;
    if (t && e->prog.w4_gru_lean)  // the lean GRU / LSTM tick: <tiles per wave, head tiles, hidden tiles per wave>
      std::snprintf(buf, cap, "%s<%d, %d, %d>", e->prog.gru.cell == 1 ? "policy_lstm_kernel" : "policy_gru_kernel", t,
                    h, e->prog.gru.H / 64);
    else if (t && e->prog.w4_plain)  // the lean pipeline kernel: <tiles per wave, head tiles, layer-0 chunks mod 4,
                                     // act, hidden layers, waves per workgroup (4)>
      std::snprintf(buf, cap, "policy_mlp_kernel<%d, %d, %d, %d, %d, 4>", t, h, c0m, e->prog.w4_actc, e->prog.w4_nhc);
    else
      std::snprintf(buf, cap, "policy_fused_kernel<%d, %d, %d, %d, %d, %d, %d>", e->waves, t, h, c0m,
                    (e->prog.has_gru && e->prog.gru.cell == 1) ? 1 : 0, t ? e->prog.w4_actc : -1,
                    t ? e->prog.w4_nhc : 0);
    return GO2PI_OK;
  });
}

int go2pi_resident_kernel(const go2pi_engine *e, char *buf, size_t cap) {
  return guarded([&] {
    check_engine(e);
    if (!buf || cap == 0) throw ApiError("null buffer", GO2PI_E_INVALID);
    const char *ring = e->req_bar_bytes ? " ring=vram" : " ring=host";
    if (!e->resident_ok) {
      std::snprintf(buf, cap, "none");
    } else if (e->resident1) {
      std::snprintf(buf, cap, "%s%s",
                    go2pi::resident1_ctl_granules(e->prog) ? "policy_act1_kernel" : "policy_resident1_kernel", ring);
    } else if (e->wide) {
      const go2pi::WideShape w = go2pi::wide_shape(e->prog);
      const bool pro = e->prog.pre_sub || e->prog.pre_div || e->prog.pre_mul || e->prog.pre_clip;
      std::snprintf(buf, cap, "policy_wide_kernel<%d, %d, %d, %d>%s", w.nl, w.cw, w.f0, pro ? 1 : 0, ring);
    } else {
      std::snprintf(buf, cap, "policy_resident_kernel%s", ring);
    }
    return GO2PI_OK;
  });
}

int go2pi_resident_launches(const go2pi_engine *e, int64_t *n) {
  return guarded([&] {
    check_engine(e);
    if (!n) throw ApiError("null argument", GO2PI_E_INVALID);
    *n = e->res_launches;
    return GO2PI_OK;
  });
}

int go2pi_inspect_model(const char *path, char *buf, size_t cap) {
  return guarded([&] {
    if (!path || !buf || cap == 0) throw ApiError("null argument", GO2PI_E_INVALID);
    std::ifstream f(path, std::ios::binary);
    if (!f) throw ApiError(std::string("cannot open model file '") + path + "'", GO2PI_E_MODEL);
    std::vector<uint8_t> bytes((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
    go2pi::Model m;
    try {
      m = go2pi::parse_onnx(bytes.data(), bytes.size());
    } catch (const std::exception &ex) {
      throw ApiError(ex.what(), GO2PI_E_MODEL);
    }
    const std::string j = go2pi::inspect_json(m);
    const size_t k = std::min(cap - 1, j.size());
    std::memcpy(buf, j.data(), k);
    buf[k] = 0;
    return (int)j.size();
  });
}

int go2pi_diag_stamps(go2pi_engine *e, uint64_t *out, int64_t n) {
  return guarded([&] {
    check_engine(e);
    if (!e->prog.stamps) throw ApiError("stamps disabled (set GO2PI_DIAG_STAMPS before create)", GO2PI_E_INVALID);
    if (!out || n < 0) throw ApiError("bad stamps buffer", GO2PI_E_INVALID);
    hip_check(hipSetDevice(e->device), "hipSetDevice");
    hip_check(hipDeviceSynchronize(), "hipDeviceSynchronize");
    const int64_t k = std::min(n, e->n_stamps);
    hip_check(hipMemcpy(out, e->prog.stamps, k * sizeof(uint64_t), hipMemcpyDeviceToHost), "hipMemcpy");
    return (int)k;
  });
}

const char *go2pi_last_error(void) { return g_last_error.c_str(); }

const char *go2pi_version(void) { return "go2pi 0.1.0 (gfx950)"; }

}  // extern "C"
