// policy_resident_kernel — the batch-1 act() path without a launch per call
// (north_star: "a persistent-kernel / hipGraph path captures one control step
// to kill launch latency at batch=1").
//
// The reference runs one onnxruntime Session::Run per control tick
// (onnx_inference/src/cpp/onnx_actor.cpp:38-48, called from
// onnx_controller/src/controller.cpp:215 every 20 ms). policy_latency_kernel
// (kernels.hip) does that tick in one launch; this kernel stays resident
// between ticks instead, so a tick costs no launch and no dispatch:
//
//  * the host writes the observation as 8-byte {epoch, value} granules into
//    pinned host-mapped memory, then a header granule {epoch, batch};
//  * wave 0 of workgroup 0 polls the header together with the first
//    observation granules in one system-scope sweep (the data IS the flag,
//    cdna_hip_programming.md Guideline 16 recipe R2), so the observation has
//    arrived when the request is seen, and mirrors the request into device
//    memory for the other workgroups (with every workgroup polling the host,
//    the 32 pollers of the 48->512^3->12 policy made a call 4.6 us SLOWER than
//    a launch per call; the shipped policy's 8 were 5 us faster);
//  * every workgroup computes all of layer 0 itself (local_layer0: no hand-off
//    for its outputs); layers 1.. run as in policy_latency_kernel (same
//    per-output summation order), with layer-l granules tagged epoch + 1 + l;
//    workgroup 0 writes the action rows to host-mapped memory and sets the
//    host-mapped done word to the epoch. (GO2PI_RES_TILED0=1: layer 0 tiled
//    too, bit-identical to the launch-per-call path.)
//
// Leaving: on a GO2PI_RES_LEAVE header, on idle_ticks of the 100 MHz wall clock
// without a request, or when a sweep meets a GO2PI_RES_LEAVE-tagged granule, a
// workgroup tags every granule slot it produces GO2PI_RES_LEAVE (so consumers
// still waiting on it leave at once instead of spinning to their bound) and
// exits; workgroup 0 sets done = GO2PI_RES_LEAVE. Every spin is bounded, so the
// grid always drains. The host relaunches on its next request.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>

#include "ctl_fn.hpp"
#include "device_fn.hpp"
#include "program.hpp"
#include "resident_fn.hpp"

namespace go2pi {

namespace {

constexpr int RES_WAVES = 8;
constexpr int RES_MAXS = 8;  // chunk slots per wave held in registers (K_pad <= 1024)
constexpr int RES_POLL = 2;  // header + observation granules per lane in the idle poll (<= 127 obs floats)
constexpr int RES_GS = 4;    // GRU form: gate-fragment chunk slots per wave (I_pad + H <= 512)
// The wave that sums a layer's partials and publishes its granules (and an RNN
// cell's h'): the last one, not wave 0, which alone sweeps the next layer's input
// at batch 1 (a wave's loads complete in order behind its own stores, so a
// publishing sweeper waits for its granule stores to be acknowledged first)
constexpr int RES_PW = RES_WAVES - 1;


// GO2PI_DIAG_RESCLK builds (tools/res_timeline.py): wall-clock (100 MHz) stamps of
// one request's path through workgroup 0 (slots 0..15) and workgroup 17 (16..31,
// another XCD), 32 per request, the last 512 requests (engine stamps buffer)
#ifdef GO2PI_DIAG_RESCLK
#define RES_STAMP(i)                                                                        \
  do {                                                                                      \
    if (P.stamps && tid == 0 && (g == 0 || g == 17))                                        \
      ((gu64_t *)P.stamps)[(size_t)(nreq & 511) * 32 + (g ? 16 : 0) + (i)] = wall_clock64();  \
  } while (0)
// shader-clock stamp beside them (slot i): the clock the request ran at
#define RES_CLOCK(i)                                                                        \
  do {                                                                                      \
    if (P.stamps && tid == 0 && (g == 0 || g == 17))                                        \
      ((gu64_t *)P.stamps)[(size_t)(nreq & 511) * 32 + (g ? 16 : 0) + (i)] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#else
#define RES_STAMP(i) \
  do {               \
  } while (0)
#define RES_CLOCK(i) \
  do {               \
  } while (0)
#endif

// One wave sweeps n granules until every tag equals `tag`: 1 done, -1 a producer
// left (GO2PI_RES_LEAVE tag), 0 timeout (err set).
template <int SCOPE>
__device__ __forceinline__ int sweep(const u64 *g, int n, unsigned tag, float *dst, unsigned *err, int lane) {
  constexpr int U = 8;
  u64 *gm = const_cast<u64 *>(g);
  for (unsigned spins = 0;; ++spins) {
    bool ok = true, leave = false;
    for (int base = 0; base < n; base += 64 * U) {
      u64 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = __hip_atomic_load(gm + min(base + u * 64 + lane, n - 1), __ATOMIC_RELAXED, SCOPE);
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int i = base + u * 64 + lane;
        if (i < n) {
          const unsigned t = (unsigned)(v[u] >> 32);
          ok &= t == tag;
          leave |= t == GO2PI_RES_LEAVE;
          dst[i] = __uint_as_float((unsigned)v[u]);
        }
      }
    }
    if (__any(leave)) return -1;
    if (__all(ok)) return 1;
    if (spins > (1u << 22)) {
      if (lane == 0) __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      return 0;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}

// Wave-level wait for the next request in `q` ([0] = {epoch, batch} header,
// [1 + i] = {epoch, obs[i]}): the header and the first observation granules are
// read in one sweep, so for a small request the observation has arrived when the
// request is seen. Leaves (leave = 1) on a GO2PI_RES_LEAVE header or idle_ticks
// of the 100 MHz wall clock without a request.
template <int SCOPE, int NP = RES_POLL>
// yield (workgroup 0 only, else null): the device's batched-launch counter (every
// batched kernel adds 1 at its start); a change since y0 means a batched kernel
// wants the CUs this kernel holds: leave (the next request relaunches).
// row1 (optional): where a one-row request's values go instead of obsv (the single-
// workgroup kernel's layer-0 input row: no staging copy when no prologue applies)
__device__ __forceinline__ void wait_request(const u64 *q, int in_dim, unsigned last, u64 idle_ticks, float *obsv,
                                             unsigned *err, int lane, int &leave, unsigned &e, int &B,
                                             unsigned &word, const unsigned *yield = nullptr, unsigned y0 = 0,
                                             float *row1 = nullptr) {
  u64 *qm = const_cast<u64 *>(q);
  const u64 t0 = wall_clock64();
  const int npoll = min(1 + in_dim, 64 * NP);
  leave = 0;
  for (;;) {
    if (yield && __hip_atomic_load(const_cast<unsigned *>(yield), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != y0) {
      leave = 1;
      return;
    }
    u64 v[NP];
#pragma unroll
    for (int u = 0; u < NP; ++u)
      if (u * 64 < npoll) v[u] = __hip_atomic_load(qm + min(u * 64 + lane, npoll - 1), __ATOMIC_RELAXED, SCOPE);
    const u64 h = __shfl(v[0], 0);
    const unsigned tag = (unsigned)(h >> 32);
    if (tag == GO2PI_RES_LEAVE) {
      leave = 1;
      return;
    }
    if (tag != 0u && tag != last) {
      e = tag;
      word = (unsigned)h;
      B = min(max((int)(word & 0xFFu), 1), GO2PI_SMALL_MAXB);
      const int n = B * in_dim;  // observation granules q[1 .. n]
      if (1 + n <= npoll) {
        bool ok = true;
        float *dst = (row1 && B == 1) ? row1 : obsv;
#pragma unroll
        for (int u = 0; u < NP; ++u) {
          const int i = u * 64 + lane;
          if (u * 64 < npoll && i >= 1 && i <= n) {
            ok &= (unsigned)(v[u] >> 32) == e;
            dst[i - 1] = __uint_as_float((unsigned)v[u]);
          }
        }
        if (__all(ok)) return;
      } else {
        if (sweep<SCOPE>(q + 1, n, e, obsv, err, lane) != 1) leave = 1;
        return;
      }
    }
    if (wall_clock64() - t0 > idle_ticks) {
      leave = 1;
      return;
    }
    __builtin_amdgcn_s_sleep(2);
  }
}

// Tag every granule this workgroup produces GO2PI_RES_LEAVE (all layers, all rows;
// a GRU policy's hidden-row granules too).
__device__ void tag_leave(const DevProgram &P, u64 *gran, int gstride, int g, int tid, int l0, u64 *hgran) {
  if (hgran && g < (P.gru.H >> 4) && tid < 2 * GO2PI_SMALL_MAXB * 16)  // both buffers
    __hip_atomic_store(hgran + (size_t)(tid >> 4) * P.gru.H + g * 16 + (tid & 15), (u64)GO2PI_RES_LEAVE << 32,
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  for (int l = l0; l + 1 < P.nl; ++l) {
    const DevLayer &L = P.L[l];
    if (g >= (L.N_pad >> 4)) continue;
    if (tid < GO2PI_SMALL_MAXB * 16) {
      const int b = tid >> 4, n = g * 16 + (tid & 15);
      __hip_atomic_store(gran + (size_t)l * gstride + b * L.N_pad + n, (u64)GO2PI_RES_LEAVE << 32, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// Layer 0 computed by EVERY workgroup for itself ("local layer 0"), so its
// outputs need no hand-off: thread tid owns output n = tid % N0 over k-chunk
// slice ks = tid / N0 (KS = 512 / N0 slices), its NF fragments held in registers
// for the kernel's life; the input rows come from LDS as broadcast float4 reads.
// One fma chain per output in k order (KS partials summed in slice order), so
// this path is deterministic but not bit-identical to the launch-per-call one.
template <int NF>
__device__ __forceinline__ void local_layer0(const DevProgram &P, const float4 (&w0)[NF], float b0, const float *obsv,
                                             float *x0, float *p0, float *xs, int B, int tid) {
  const DevLayer &L = P.L[0];
  // x0 rows hold NF / 4 chunks per slice (zero-padded past layer 0's own chunks)
  const int N0 = L.N_pad, KS = (RES_WAVES * 64) / N0, K0 = (NF / 4) * KS * 16;
  for (int i = tid; i < B * K0; i += RES_WAVES * 64) {
    const int b = i / K0, k = i - b * K0;
    x0[i] = k < P.in_dim ? prologue(P, obsv[b * P.in_dim + k], k) : 0.f;
  }
  lds_barrier();
  const int n = tid % N0, ks = tid / N0;
  const int K1 = P.L[1].K_pad;  // layer 1's input row stride (= N0)
  for (int b = 0; b < B; ++b) {
    float acc = 0.f;
#pragma unroll
    for (int f = 0; f < NF; ++f) {
      // fragment f: chunk c = ks + KS * (f >> 2), quad q = f & 3 -> k = 16c + 4q .. +3
      const int k = 16 * (ks + KS * (f >> 2)) + 4 * (f & 3);
      const float4 a = *reinterpret_cast<const float4 *>(x0 + b * K0 + k);
      acc = fmaf(a.x, w0[f].x, acc);
      acc = fmaf(a.y, w0[f].y, acc);
      acc = fmaf(a.z, w0[f].z, acc);
      acc = fmaf(a.w, w0[f].w, acc);
    }
    if (KS == 1) {
      xs[b * K1 + n] = act_fn(L.act, L.alpha, L.beta, acc + b0);
    } else {
      p0[(ks * GO2PI_SMALL_MAXB + b) * N0 + n] = acc;
    }
  }
  if (KS > 1) {
    lds_barrier();
    for (int i = tid; i < B * N0; i += RES_WAVES * 64) {
      const int b = i / N0, nn = i - b * N0;
      float acc = 0.f;
      for (int s2 = 0; s2 < KS; ++s2) acc += p0[(s2 * GO2PI_SMALL_MAXB + b) * N0 + nn];
      xs[b * K1 + nn] = act_fn(L.act, L.alpha, L.beta, acc + L.bias[nn]);
    }
  }
  lds_barrier();
}

}  // namespace

// NF > 0: local layer 0 (above) with NF fragments per thread; 0: layer 0 tiled
// over the workgroups like every other layer (policy_latency_kernel's order).
// CTL: the controller tick (go2pi_controller_step at batch <= 8): workgroup 0
// reads the tick's raw rows from the host staging named by `C` once the header
// arrives, assembles the observation (ctl_fn.hpp, as policy_latency_ctl_kernel),
// mirrors it, and post-processes the action into the staging (ctl_store); the
// header's low word carries the batch and GO2PI_RES_* flags.
//
// RNN: 1 a GRU policy (ONNX GRU, linear_before_reset = 1, H % 64 == 0), 2 an LSTM
// policy (ONNX LSTM, gates i, o, f, c; no peepholes). The cell runs as a tiled
// layer in front of the dense ones: workgroup g < H / 16 owns hidden units
// [16g, 16g + 16), its gate fragments held in registers for the kernel's life; it
// computes the gates over [x | h] by GEMV (8 waves split the k-chunks, fixed-order
// reductions) and publishes h' as {epoch, value} granules. An LSTM's cell state
// never leaves the workgroup that owns its units: it lives in that workgroup's LDS
// between requests (first read from the engine's state rows, written back on leave).
// Those granules ARE the carried hidden state: dense layer 0 sweeps them as its
// input (tag = this request's epoch), and the next request's cell sweeps them as
// its h (tag = the epoch of the last request that covered that row). Every
// workgroup tracks, per row, that epoch and which of two granule buffers
// (hgran [2][8][H]) holds it, identically (all see the same requests): h' is
// written to the OTHER buffer, because the request's other cell workgroups are
// still reading the row's current h from this one (an in-place update raced
// them). A row not yet written in this launch comes from the engine's state rows
// in HBM; each cell workgroup writes its units' latest h' back to those rows when
// the kernel leaves (not while it runs: the rows are read then).
template <int NF, bool CTL, int RNN = 0>
__global__ __launch_bounds__(RES_WAVES * 64) void policy_resident_kernel(const DevProgram *__restrict__ Pd,
                                                                         const u64 *req, u64 *actg, u64 *gran,
                                                                         int gstride, u64 *mirror, unsigned *err,
                                                                         unsigned *done, u64 idle_ticks, DevCtl C,
                                                                         u64 *hgran, float *hidden,
                                                                         const unsigned *yield) {
  static_assert(!(RNN && (NF > 0 || CTL)), "the GRU form tiles layer 0 and serves act() only");
  constexpr bool LOCAL0 = NF > 0;
  constexpr bool LSTM = RNN == 2;
  constexpr int NG = LSTM ? 4 : 3;  // gate fragments per (chunk, tile)
  const DevProgram &P = *Pd;
  extern __shared__ float4 lds4[];
  float *xs = reinterpret_cast<float *>(lds4);                       // [B][K_pad] layer input
  float *part = xs + GO2PI_SMALL_MAXB * P.lds_stride;                // [waves][B][16] partial sums
  int *st = reinterpret_cast<int *>(part + RES_WAVES * GO2PI_SMALL_MAXB * 16);  // [0] leave, [1] epoch, [2] batch
  float *obsv = reinterpret_cast<float *>(st + 4);                   // [B][in_dim] the request's observation
  float *x0 = obsv + GO2PI_SMALL_MAXB * P.in_dim;                    // LOCAL0: [B][K0] prologued layer-0 input
  // LOCAL0: x0 rows of NF / 4 chunks per k-slice (>= K_pad), then the KS > 1 partials [KS][B][N0]
  const int x0len = LOCAL0 ? (NF / 4) * ((RES_WAVES * 64) / P.L[0].N_pad) * 16 : P.L[0].K_pad;
  float *p0 = x0 + GO2PI_SMALL_MAXB * x0len;
  // CTL: the LDS image of the tick's inputs (16-byte aligned: q0 is double)
  // (p0's size: KS * MAXB * N0 floats when 512 / N0 = KS > 1 slices, as launch_resident reserves)
  const int ks0 = ((RES_WAVES * 64) % P.L[0].N_pad == 0 && P.L[0].N_pad < RES_WAVES * 64) ? (RES_WAVES * 64) / P.L[0].N_pad : 0;
  float *cbase = p0 + (ks0 * GO2PI_SMALL_MAXB * P.L[0].N_pad + 3) / 4 * 4;
  const CtlLds CL = ctl_lds(cbase, GO2PI_SMALL_MAXB, P.in_dim);
  float *craw = cbase + ctl_lds_floats(GO2PI_SMALL_MAXB, P.in_dim);  // CTL: [B][GO2PI_CTL_RAW + in_dim] request rows
  const int g = blockIdx.x, tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int in_dim = P.in_dim;
  unsigned last = 0;
  unsigned nreq = 0;  // requests served by this launch (diagnostic stamps)
  (void)nreq;
  // the batched-launch counter at launch (workgroup 0 leaves when it moves)
  const unsigned y0 =
      (g == 0 && yield) ? __hip_atomic_load(const_cast<unsigned *>(yield), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
  // RNN: the cell's LDS (after the CTL regions: RNN and CTL are exclusive)
  const int Hh = RNN ? P.gru.H : 0, Ip = RNN ? P.gru.I_pad : 0, Kg = Ip + Hh, Cg = Kg >> 4, Cx = Ip >> 4;
  const int SW = RNN ? P.gru.sw : 0;  // state floats per robot row (LSTM: h | c)
  const int Ht = Hh >> 4;
  float *hx = cbase;                                      // [B][Kg] the cell's input rows [x | h]
  float *hpart = hx + GO2PI_SMALL_MAXB * Kg;              // [waves][4][B][16] partial sums (z, r, n_x, n_h)
  unsigned *le = reinterpret_cast<unsigned *>(hpart + RES_WAVES * 4 * GO2PI_SMALL_MAXB * 16);  // [B] row epochs
  unsigned *lb = le + GO2PI_SMALL_MAXB;                   // [B] the granule buffer holding each row's h
  float *hown = reinterpret_cast<float *>(lb + GO2PI_SMALL_MAXB);  // [B][16] this workgroup's units' latest h'
  float *cown = hown + GO2PI_SMALL_MAXB * 16;             // LSTM: [B][16] its units' cell state
  // the cell's outputs of the request in flight, copied to hown / cown only once this
  // workgroup has finished the request: a request abandoned mid-layers (a sweep met a
  // LEAVE tag) then leaves the committed state, which the leave path writes back, as it was
  float *hst = cown + GO2PI_SMALL_MAXB * 16;              // [B][16]
  float *cst = hst + GO2PI_SMALL_MAXB * 16;               // LSTM: [B][16]
  const size_t hbuf = (size_t)GO2PI_SMALL_MAXB * Hh;      // granules per buffer
  float4 wgf[RES_GS][NG];                                 // this workgroup's gate fragments (chunks wave + 8s)
  float gb[4] = {0.f, 0.f, 0.f, 0.f};                     // its biases: GRU z, r (summed), Wb_h, Rb_h; LSTM i, o, f, c
  if constexpr (RNN) {
    if (tid < GO2PI_SMALL_MAXB) le[tid] = lb[tid] = 0u;
    if (g < Ht) {
      const float4 *Wg = reinterpret_cast<const float4 *>(P.gru.w);
#pragma unroll
      for (int s = 0; s < RES_GS; ++s) {
        const int c = wave + s * RES_WAVES;
#pragma unroll
        for (int q = 0; q < NG; ++q)
          wgf[s][q] = c < Cg ? Wg[(((size_t)c * Ht + g) * NG + q) * 64 + lane] : make_float4(0.f, 0.f, 0.f, 0.f);
      }
      if (wave == RES_PW && lane < 16) {
        const int j = g * 16 + lane;
        if constexpr (LSTM) {  // Wb + Rb per gate, summed at load
#pragma unroll
          for (int q = 0; q < 4; ++q) gb[q] = P.gru.bzr[q * Hh + j];
        } else {
          gb[0] = P.gru.bzr[j];
          gb[1] = P.gru.bzr[Hh + j];
          gb[2] = P.gru.bh[j];
          gb[3] = P.gru.bh[Hh + j];
        }
      }
    }
  }
  // The weight fragments of the next layer this workgroup owns a tile of are
  // loaded one layer ahead, and those of its first layer before each request
  // wait, so a request meets them in registers (the launch-per-call kernel
  // fetches layer 0's from L2 after its launch).
  auto owned_from = [&](int l) {
    if (LOCAL0 && l == 0) l = 1;  // layer 0 has its own registers (w0)
    while (l < P.nl && g >= (P.L[l].N_pad >> 4)) ++l;
    return l;  // P.nl: none
  };
  float4 wr[RES_MAXS];
  float bv = 0.f;
  auto load_layer = [&](int l) {
    const DevLayer &L = P.L[l];
    const int T = L.N_pad >> 4, C = L.K_pad >> 4;
    const float4 *W = reinterpret_cast<const float4 *>(L.w) + (size_t)g * 64 + lane;
#pragma unroll
    for (int s = 0; s < RES_MAXS; ++s) {
      const int c = wave + s * RES_WAVES;
      wr[s] = c < C ? W[(size_t)c * T * 64] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    bv = (wave == RES_PW && lane < 16) ? L.bias[g * 16 + lane] : 0.f;
  };
  const int l_first = owned_from(0);
  if (l_first < P.nl) load_layer(l_first);
  float4 w0[LOCAL0 ? NF : 1];
  float b0 = 0.f;
  if constexpr (LOCAL0) {
    const DevLayer &L = P.L[0];
    const int N0 = L.N_pad, KS = (RES_WAVES * 64) / N0, n = tid % N0, ks = tid / N0;
    const float4 *W = reinterpret_cast<const float4 *>(L.w);
#pragma unroll
    for (int f = 0; f < NF; ++f) {
      const int c = ks + KS * (f >> 2), q = f & 3;  // (chunks past layer 0's: zero fragments)
      w0[f] = c < (L.K_pad >> 4) ? W[((size_t)c * (N0 >> 4) + (n >> 4)) * 64 + (n & 15) + 16 * q]
                                 : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    b0 = L.bias[n];
  }
  // every fragment held across requests has landed before the first wait (and the
  // compiler's waitcnt pass knows it: no vmcnt(0) in front of their first uses,
  // which would also wait for the stores a request has in flight by then)
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)

  for (;;) {
    // ---- wait for a request. Workgroup 0 polls the host (header + the first
    // observation granules in one sweep) and mirrors the request into device
    // memory; the others poll that mirror, so one wave, not the grid, reads
    // host memory over PCIe while idle.
    if (wave == 0) {
      int leave = 0, B = 0;
      unsigned e = 0, word = 0;
      if (g == 0) {
        // CTL: the header with the tick's rows as tagged granules (3 per lane per poll:
        // one robot's 53 + in_dim floats arrive with the request); act: the observation
        if constexpr (CTL)
          wait_request<__HIP_MEMORY_SCOPE_SYSTEM, 3>(req, GO2PI_CTL_RAW + in_dim, last, idle_ticks, craw, err, lane,
                                                     leave, e, B, word, yield, y0);
        else
          wait_request<__HIP_MEMORY_SCOPE_SYSTEM>(req, in_dim, last, idle_ticks, obsv, err, lane, leave, e, B, word,
                                                  yield, y0);
        RES_STAMP(0);
        const int n = (leave || CTL) ? 0 : B * in_dim;
        for (int i = lane; i < n; i += 64)
          __hip_atomic_store(mirror + 1 + i, ((u64)e << 32) | __float_as_uint(obsv[i]), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
        if (lane == 0 && (leave || !CTL))
          __hip_atomic_store(mirror, leave ? ((u64)GO2PI_RES_LEAVE << 32) : (((u64)e << 32) | (unsigned)B),
                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        RES_STAMP(1);
      } else {
        wait_request<__HIP_MEMORY_SCOPE_AGENT>(mirror, in_dim, last, idle_ticks, obsv, err, lane, leave, e, B, word);
        RES_STAMP(0);
      }
      if (lane == 0) {
        st[0] = leave;
        st[1] = (int)e;
        st[2] = B;
        st[3] = (int)word;
      }
    }
    lds_barrier();  // (the mirror stores stay in flight)
    if (st[0]) break;
    RES_STAMP(2);
    RES_CLOCK(15);
    const unsigned e = (unsigned)st[1];
    const int B = st[2];
    const unsigned word = (unsigned)st[3];
    last = e;
    bool left = false;
    bool refill = false;  // this workgroup's last layer ran: its first layer's fragments are due
    CtlView cv{};
    if constexpr (CTL) {
      if (g == 0) {
        // the request's rows (craw: state | joystick | previous obs | previous action, each
        // B rows) into the assembly's LDS image
        const bool joy = (word & GO2PI_RES_JOY) != 0u;
        const int o_jy = B * GO2PI_CTL_STATE_DIM, o_obs = o_jy + B * GO2PI_CTL_JOY_DIM, o_act = o_obs + B * in_dim;
        for (int i = tid; i < o_jy; i += RES_WAVES * 64) CL.st[i] = craw[i];
        for (int i = tid; i < B * GO2PI_CTL_JOY_DIM; i += RES_WAVES * 64) CL.jy[i] = craw[o_jy + i];
        for (int i = tid; i < B * in_dim; i += RES_WAVES * 64) CL.obs[i] = craw[o_obs + i];
        for (int i = tid; i < B * GO2PI_CTL_DOF; i += RES_WAVES * 64) CL.act[i] = craw[o_act + i];
        if (tid < GO2PI_CTL_DOF) CL.q0[tid] = C.prm->q0[tid];
        if (tid < GO2PI_TILE_ROWS) CL.nanf[tid] = 0u;
        __syncthreads();
        ctl_assemble_flat<false, 4>(P, CL, ctl_q(P, C), joy, B, obsv, in_dim, nullptr, tid, RES_WAVES * 64);
        __syncthreads();
        if (wave == 0) {  // mirror the assembled observation for the other workgroups
          for (int i = lane; i < B * in_dim; i += 64)
            __hip_atomic_store(mirror + 1 + i, ((u64)e << 32) | __float_as_uint(obsv[i]), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
          if (lane == 0)
            __hip_atomic_store(mirror, ((u64)e << 32) | (unsigned)B, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        DevCtl c = C;
        if (!joy) c.joy = nullptr;
        if (!(word & GO2PI_RES_QDES)) c.q_des = nullptr;
        if (!(word & GO2PI_RES_KP)) c.kp = nullptr;
        if (!(word & GO2PI_RES_KD)) c.kd = nullptr;
        cv = ctl_view(c, CL, 0);
      }
    }

    // ---- RNN: the GRU cell (tiled; h' as granules tagged e, and to the state rows)
    if constexpr (RNN) {
      if (g < Ht) {
        for (int i = tid; i < B * Ip; i += RES_WAVES * 64) {
          const int b = i / Ip, k = i - b * Ip;
          hx[b * Kg + k] = k < in_dim ? prologue(P, obsv[b * in_dim + k], k) : 0.f;
        }
        if (wave < B) {  // wave b gathers row b's h: this launch's granules, else the state row
          const int b = wave;
          const unsigned te = le[b];
          if (te != 0u) {
            if (sweep<__HIP_MEMORY_SCOPE_AGENT>(hgran + lb[b] * hbuf + (size_t)b * Hh, Hh, te, hx + b * Kg + Ip, err,
                                                lane) != 1 &&
                lane == 0)
              st[0] = 1;
          } else {
            for (int k = lane; k < Hh; k += 64) hx[b * Kg + Ip + k] = hidden[(size_t)b * SW + k];
          }
        }
        __syncthreads();
        if (st[0]) left = true;
#ifdef GO2PI_DIAG_RESDBG
        if (tid == 0) printf("g %d e %u B %d gru staged left %d le0 %u hx %g %g\n", g, e, B, (int)left, le[0], hx[0], hx[Ip]);
#endif
        if (!left) {
          float pz[GO2PI_SMALL_MAXB], pr[GO2PI_SMALL_MAXB], pnx[GO2PI_SMALL_MAXB], pnh[GO2PI_SMALL_MAXB];
#pragma unroll
          for (int b = 0; b < GO2PI_SMALL_MAXB; ++b) pz[b] = pr[b] = pnx[b] = pnh[b] = 0.f;
          const int koff = (lane >> 4) << 2;
          auto dot4 = [](const float4 &a, const float4 &w, float acc) {
            acc = fmaf(a.x, w.x, acc);
            acc = fmaf(a.y, w.y, acc);
            acc = fmaf(a.z, w.z, acc);
            return fmaf(a.w, w.w, acc);
          };
#pragma unroll
          for (int s = 0; s < RES_GS; ++s) {
            const int c = wave + s * RES_WAVES;
            if (c >= Cg) break;
            const bool xc = c < Cx;
#pragma unroll
            for (int b = 0; b < GO2PI_SMALL_MAXB; ++b) {
              if (b < B) {
                const float4 a = *reinterpret_cast<const float4 *>(hx + b * Kg + c * 16 + koff);
                pz[b] = dot4(a, wgf[s][0], pz[b]);  // LSTM: i, o, f, c in pz, pr, pnx, pnh
                pr[b] = dot4(a, wgf[s][1], pr[b]);
                if constexpr (LSTM) {
                  pnx[b] = dot4(a, wgf[s][2], pnx[b]);
                  pnh[b] = dot4(a, wgf[s][NG - 1], pnh[b]);
                } else {
                  if (xc) pnx[b] = dot4(a, wgf[s][2], pnx[b]);
                  else pnh[b] = dot4(a, wgf[s][2], pnh[b]);
                }
              }
            }
          }
#pragma unroll
          for (int b = 0; b < GO2PI_SMALL_MAXB; ++b) {
            pz[b] += __shfl_xor(pz[b], 16);
            pz[b] += __shfl_xor(pz[b], 32);
            pr[b] += __shfl_xor(pr[b], 16);
            pr[b] += __shfl_xor(pr[b], 32);
            pnx[b] += __shfl_xor(pnx[b], 16);
            pnx[b] += __shfl_xor(pnx[b], 32);
            pnh[b] += __shfl_xor(pnh[b], 16);
            pnh[b] += __shfl_xor(pnh[b], 32);
          }
          if (lane < 16) {
#pragma unroll
            for (int b = 0; b < GO2PI_SMALL_MAXB; ++b) {
              if (b < B) {
                float *hp = hpart + ((size_t)wave * 4 * GO2PI_SMALL_MAXB + b) * 16 + lane;
                hp[0] = pz[b];
                hp[GO2PI_SMALL_MAXB * 16] = pr[b];
                hp[2 * GO2PI_SMALL_MAXB * 16] = pnx[b];
                hp[3 * GO2PI_SMALL_MAXB * 16] = pnh[b];
              }
            }
          }
          __syncthreads();
          if (wave == RES_PW && lane < 16) {
            const int j = g * 16 + lane;
            for (int b = 0; b < B; ++b) {
              float q[4];
#pragma unroll
              for (int k = 0; k < 4; ++k) {
                float a = 0.f;
                for (int w2 = 0; w2 < RES_WAVES; ++w2) a += hpart[((w2 * 4 + k) * GO2PI_SMALL_MAXB + b) * 16 + lane];
                q[k] = a + gb[k];
              }
              float hnew;
              if constexpr (LSTM) {  // the gate math of lstm_group (fused_impl.hpp)
                const float ig = sigmoid_fast(q[0]), og = sigmoid_fast(q[1]), fg = sigmoid_fast(q[2]);
                const float cg = 2.f * sigmoid_fast(2.f * q[3]) - 1.f;  // tanh, ~1e-7 abs
                // c: this workgroup's LDS copy once the row ran in this launch, else the state row
                const float c_old = le[b] != 0u ? cown[b * 16 + lane] : hidden[(size_t)b * SW + Hh + j];
                const float c_new = fg * c_old + ig * cg;
                cst[b * 16 + lane] = c_new;
                hnew = og * (2.f * sigmoid_fast(2.f * c_new) - 1.f);
              } else {
                const float zg = sigmoid_fast(q[0]), rg = sigmoid_fast(q[1]);
                const float hv = 2.f * sigmoid_fast(2.f * (q[2] + rg * q[3])) - 1.f;  // tanh, ~1e-7 abs
                hnew = (1.f - zg) * hv + zg * hx[b * Kg + Ip + j];
              }
              hst[b * 16 + lane] = hnew;
              __hip_atomic_store(hgran + (1u - lb[b]) * hbuf + (size_t)b * Hh + j, ((u64)e << 32) | __float_as_uint(hnew),
                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
          }
        }
      }
      if (left) break;
    }
    // ---- the layers (policy_latency_kernel's body; tags e + 1 + l)
    if constexpr (LOCAL0) local_layer0<NF>(P, w0, b0, obsv, x0, p0, xs, B, tid);
    RES_STAMP(3);
    for (int l = LOCAL0 ? 1 : 0; l < P.nl; ++l) {
      const DevLayer &L = P.L[l];
      const int T = L.N_pad >> 4, C = L.K_pad >> 4, K_pad = L.K_pad;
      if (g >= T) continue;  // this workgroup owns no tile of layer l
      // wr / bv hold layer l (prefetched)
      if (l == 0 && RNN) {  // the GRU's h' granules (tag e; row b in buffer 1 - lb[b]), [B][H] = [B][K_pad]
        if (wave < B && sweep<__HIP_MEMORY_SCOPE_AGENT>(hgran + (1u - lb[wave]) * hbuf + (size_t)wave * Hh, Hh, e,
                                                        xs + wave * K_pad, err, lane) != 1 &&
            lane == 0)
          st[0] = 1;
      } else if (l == 0) {
        for (int i = tid; i < B * K_pad; i += RES_WAVES * 64) {
          const int b = i / K_pad, k = i - b * K_pad;
          xs[i] = k < in_dim ? prologue(P, obsv[b * in_dim + k], k) : 0.f;
        }
      } else if (!(LOCAL0 && l == 1)) {  // (local layer 0 left layer 1's input in xs)
        // every wave sweeps its own 512 granules (8 per lane, all in flight): at
        // batch 8 one wave's eight serial rounds cost ~20 us per call
        const int n = B * K_pad, lo = wave * 512;
        if (lo < n &&
            sweep<__HIP_MEMORY_SCOPE_AGENT>(gran + (size_t)(l - 1) * gstride + lo, min(512, n - lo), e + (unsigned)l,
                                            xs + lo, err, lane) != 1 &&
            lane == 0)
          st[0] = 1;
      }
      __syncthreads();
#ifdef GO2PI_DIAG_RESDBG
      if (tid == 0 && (g == 0 || g == 20)) printf("g %d e %u layer %d input ready st0 %d xs %g\n", g, e, l, st[0], xs[0]);
#endif
      if (st[0]) {
        left = true;
        break;
      }
      if (l < 5) RES_STAMP(2 * l + 2);  // layer l's input ready
      float p[GO2PI_SMALL_MAXB];
#pragma unroll
      for (int b = 0; b < GO2PI_SMALL_MAXB; ++b) p[b] = 0.f;
      const int koff = (lane >> 4) << 2;
#pragma unroll
      for (int s = 0; s < RES_MAXS; ++s) {
        const int c = wave + s * RES_WAVES;
        if (c >= C) break;
#pragma unroll
        for (int b = 0; b < GO2PI_SMALL_MAXB; ++b) {
          if (b < B) {
            const float4 a = *reinterpret_cast<const float4 *>(xs + b * K_pad + c * 16 + koff);
            p[b] = fmaf(a.x, wr[s].x, p[b]);
            p[b] = fmaf(a.y, wr[s].y, p[b]);
            p[b] = fmaf(a.z, wr[s].z, p[b]);
            p[b] = fmaf(a.w, wr[s].w, p[b]);
          }
        }
      }
      if (l == 1) RES_STAMP(10);  // layer 1: fma chains done
      // the four 16-lane row groups' partials summed (rows past the request's batch skipped:
      // each cross-lane step is an LDS-latency permute)
#pragma unroll
      for (int b = 0; b < GO2PI_SMALL_MAXB; ++b) {
        if (b < B) {
          p[b] += __shfl_xor(p[b], 16);
          p[b] += __shfl_xor(p[b], 32);
        }
      }
      if (lane < 16) {
#pragma unroll
        for (int b = 0; b < GO2PI_SMALL_MAXB; ++b)
          if (b < B) part[(wave * GO2PI_SMALL_MAXB + b) * 16 + lane] = p[b];
      }
      if (l == 1) RES_STAMP(12);  // layer 1: partial sums written
      const float bcur = bv;
      // the next owned layer's fragments, in flight across the barriers and the next
      // hand-off; after this workgroup's last layer, the next request's first layer
      // is fetched once the request is answered (not in front of the action's drain)
      const int ln = owned_from(l + 1);
      if (ln < P.nl) load_layer(ln);
      lds_barrier();
      if (l == 1) RES_STAMP(13);  // layer 1: partials visible
      if (wave == RES_PW && lane < 16) {
        const int n = g * 16 + lane;
        const bool lastl = l == P.nl - 1;
        const int la = L.act, LN = L.N, LNP = L.N_pad;  // (read once: the stores below would make each row reload them)
        const float lal = L.alpha, lbe = L.beta;
        const Post po = post_of(P);
        for (int b = 0; b < B; ++b) {
          float s = 0.f;
          for (int w2 = 0; w2 < RES_WAVES; ++w2) s += part[(w2 * GO2PI_SMALL_MAXB + b) * 16 + lane];
          const float v = act_fn(la, lal, lbe, s + bcur);
          if (lastl) {
            if constexpr (CTL) {
              if (n < LN) ctl_store(cv, b, n, post_fn(po, v));
            } else if (n < LN) {
              // the action as {epoch, value} granules in host memory: the host's spin reads
              // the data itself (no release drain, no done word behind it)
              __hip_atomic_store(actg + (size_t)b * LN + n, ((u64)e << 32) | __float_as_uint(post_fn(po, v)),
                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
          } else {
            const u64 gv = ((u64)(e + 1u + (unsigned)l) << 32) | __float_as_uint(v);
            __hip_atomic_store(gran + (size_t)l * gstride + b * LNP + n, gv, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
          }
        }
      }
      if (l == 1) RES_STAMP(14);  // layer 1: wave 0's granules stored
      lds_barrier();  // xs / part reused by the next layer
      if (l < 5) RES_STAMP(2 * l + 3);  // layer l published (the last: done written)
      if (l == 2) RES_CLOCK(11);
      if (ln >= P.nl) refill = true;
    }
    if (left) break;
    if constexpr (RNN) {  // rows [0, B) now carry this request's h' (granules tagged e, in the other buffer)
      __syncthreads();     // every wave is done with lb for this request
      if (tid < B) {
        le[tid] = e;
        lb[tid] = 1u - lb[tid];
      }
      if (g < Ht && tid < B * 16) {  // this workgroup's units: the request is committed
        hown[tid] = hst[tid];
        if constexpr (LSTM) cown[tid] = cst[tid];
      }
    }
    if constexpr (CTL) {
      if (g == 0) {  // the new observation rows and NaN flags, then the done word
        for (int i = tid; i < B * in_dim; i += RES_WAVES * 64) C.obs[i] = obsv[i];
        if ((word & GO2PI_RES_STATUS) && tid < B) C.status[tid] = CL.nanf[tid];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) __hip_atomic_store(done, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
    // the next request's first-layer fragments, after this one is answered (they
    // land while the next request is awaited)
    if (refill && l_first < P.nl) {
      load_layer(l_first);
      // drained here, in the idle time before the next request (the builtin, unlike an
      // asm wait, tells the compiler's waitcnt pass: the next request's first use of
      // these registers then waits for nothing, not for every store issued since)
      __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
    }
    ++nreq;
  }
  // ---- leave: consumers still waiting on this workgroup's slots leave too
  tag_leave(P, gran, gstride, g, tid, LOCAL0 ? 1 : 0, RNN ? hgran : nullptr);
  if constexpr (RNN) {  // the rows this launch advanced go back to the engine's state rows
    __syncthreads();
    if (g < Ht && tid < GO2PI_SMALL_MAXB * 16 && le[tid >> 4] != 0u) {
      hidden[(size_t)(tid >> 4) * SW + g * 16 + (tid & 15)] = hown[tid];
      if constexpr (LSTM) hidden[(size_t)(tid >> 4) * SW + Hh + g * 16 + (tid & 15)] = cown[tid];
    }
  }
  if (g == 0 && tid == 0)
    __hip_atomic_store(mirror, (u64)GO2PI_RES_LEAVE << 32, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  // every wave's stores (wave RES_PW's answer granules among them) drained before the
  // LEAVE done word: a host that sees LEAVE and rescans finds a served request's answer
  // (engine.cpp resident_serve)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (g == 0 && tid == 0) __hip_atomic_store(done, GO2PI_RES_LEAVE, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// ---------------------------------------------------------------------------
// policy_resident1_kernel — the resident act() in ONE workgroup (r04), for dense
// policies whose weights fit one CU's registers: the shipped 98->128^3->12 model is
// 47,244 parameters (189 KB); a CU holds 512 KB of VGPRs. The multi-workgroup form
// above spends most of a batch-1 request on hops between workgroups (mirror 1.0 us,
// each layer hand-off 1.2 us: profiles/r03_res_timeline.json); here every layer is
// an in-workgroup reduction behind one s_barrier, with no granule, no mirror and no
// other CU involved:
//
//  * 16 waves; dense layer l gives each output n a group of G_l adjacent lanes of
//    one wave (G_l = the largest power of two with N_pad * G_l <= the threads, at
//    most 64), lane s of the group owns the input float4s k4 = s + G_l * f, f <
//    F_l <= r1_fmax(threads). Those F_l weight float4s sit in the lane's registers for the
//    kernel's life (loaded once from the packed fragments, program.hpp);
//  * per request and row: F_l broadcast ds_read_b128 of the input row, 4 F_l fmas
//    in two chains, the group's sum by DPP row permutes (quad xor 1, quad xor 2,
//    half-row mirror, row mirror, then cross-row shuffles for G > 16), and the
//    group's lane 0 adds the bias, applies the activation and writes the output
//    to the other LDS row buffer; one lds_barrier per layer;
//  * the final layer runs on waves 1..15 only, so wave 0 — the one that polls the
//    host for the next request — has no PCIe store of the answer in flight ahead of
//    its poll loads (a wave's memory ops complete in order);
//  * the request / answer protocol is the multi-workgroup form's: wave 0 polls the
//    header and observation granules in pinned host memory (wait_request), the
//    answer goes back as {epoch, value} action granules the host checks itself.
// Summation order: per output, two fma chains over its lane's k (f even / odd),
// then the fixed DPP tree over the group: deterministic, not bit-identical to the
// launch path's MFMA order (both within the 1e-5 contract of the fp64 oracle).
constexpr int R1_LMAX = 4;  // dense layers
// threads: 1024 (16 waves, 128 registers each) for act(); the controller form runs 512
// (8 waves, 256 registers each: the assembly's registers beside the weights spilled to
// scratch at 1024), twice the weight float4s per lane
__host__ __device__ constexpr int r1_fmax(int nt) { return nt >= 1024 ? 4 : 8; }

// lanes per output for a layer of n_pad outputs over `threads` lanes (at most 16: a
// group's sum then stays within a DPP row, no cross-row permute through LDS)
__host__ __device__ constexpr int r1_group(int n_pad, int threads) {
  int g = 16;
  while (g > 1 && n_pad * g > threads) g >>= 1;
  return g;
}

// a uniform value kept in an SGPR as it is (opaque to the optimizer: never reloaded)
__device__ __forceinline__ int r1_keep(int v) {
  v = __builtin_amdgcn_readfirstlane(v);
  asm volatile("" : "+s"(v));
  return v;
}
__device__ __forceinline__ float r1_keep(float v) { return __int_as_float(r1_keep(__float_as_int(v))); }

template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, false));
}

// sum over the aligned group of G lanes (G a power of two <= 64); every lane of the
// group gets the total
__device__ __forceinline__ float r1_group_sum(float v, int G) {
  if (G >= 2) v += dpp_f<0xB1>(v);   // quad_perm [1, 0, 3, 2]: lane ^ 1
  if (G >= 4) v += dpp_f<0x4E>(v);   // quad_perm [2, 3, 0, 1]: lane ^ 2
  if (G >= 8) v += dpp_f<0x141>(v);  // row_half_mirror: the other quad of the 8
  if (G >= 16) v += dpp_f<0x140>(v); // row_mirror: the other 8 of the row
  if (G >= 32) v += __shfl_xor(v, 16);
  if (G >= 64) v += __shfl_xor(v, 32);
  return v;
}

// the per-layer float4 counts of program p, packed as the kernel's FS
unsigned r1_shape(const DevProgram &p, int nt) {
  unsigned fs = 0;
  for (int l = 0; l < p.nl && l < R1_LMAX; ++l) {
    const int thr = l == p.nl - 1 ? nt - 64 : nt;
    const int G = r1_group(p.L[l].N_pad, thr);
    fs |= (unsigned)((p.L[l].K_pad + 4 * G - 1) / (4 * G)) << (4 * l);
  }
  return fs;
}

// the activation kind of each layer of program p, packed as the kernel's AS
unsigned r1_acts(const DevProgram &p) {
  unsigned as = 0;
  for (int l = 0; l < p.nl && l < R1_LMAX; ++l) as |= (unsigned)(p.L[l].act & 15) << (4 * l);
  return as;
}

// log2 of the group size of each layer of program p, packed as the kernel's GS
unsigned r1_lgs(const DevProgram &p, int nt) {
  unsigned gs = 0;
  for (int l = 0; l < p.nl && l < R1_LMAX; ++l)
    gs |= (unsigned)__builtin_ctz(r1_group(p.L[l].N_pad, l == p.nl - 1 ? nt - 64 : nt)) << (4 * l);
  return gs;
}

// the act1 shape of program p: {NL, H, F0}, or NL = 0 when it does not apply
// (policy_act1_kernel below, r05)
struct A1Shape {
  int nl, h, f0;
};
A1Shape act1_shape(const DevProgram &p);

bool resident1_fits(const DevProgram &p, bool ctl) {
  if (act1_shape(p).nl && !std::getenv("GO2PI_RES_R1W")) return true;  // policy_act1_kernel (r05)
  const int nt = ctl ? 512 : 1024;
  // (nl >= 2: with one layer nothing would separate the request loop's top barrier from
  // the polling wave's next writes of st / x0)
  if (p.has_gru || p.nl < 2 || p.nl > R1_LMAX || p.L[p.nl - 1].N_pad != 16) return false;
  for (int l = 0; l < p.nl; ++l) {
    const int thr = l == p.nl - 1 ? nt - 64 : nt;
    const int G = r1_group(p.L[l].N_pad, thr);
    if (p.L[l].N_pad * G > thr) return false;
    if ((p.L[l].K_pad + 4 * G - 1) / (4 * G) > r1_fmax(nt)) return false;
  }
  return p.L[0].K_pad <= nt;
}

bool resident1_ctl_granules(const DevProgram &p) { return act1_shape(p).nl && !std::getenv("GO2PI_RES_R1W"); }

// CTL: the controller tick (go2pi_controller_step at batch <= 8), as the multi-
// workgroup kernel's controller form: the request carries the tick's raw rows
// (state | joystick | previous obs | previous action, as tagged granules), the
// observation is assembled here (ctl_fn.hpp), the action post-processed into the
// pinned staging C names (ctl_store), the new observation rows and NaN flags written,
// then the done word.
// FS: weight float4s per lane of each layer, packed as 4-bit fields (layer l in bits
// 4l..4l+3), so a policy shape gets exactly the registers its layers need (the
// shipped model: 4, 4, 4, 1); the generic instantiation holds FMAX for every layer.
// GS: log2 of each layer's group size, packed the same way (the shipped model: 3, 3,
// 3, 5), or 0: computed at run time. At compile time every lane index is a shift and
// every input offset an immediate: with 16 waves sharing 4 SIMDs a layer is VALU-issue
// bound, and the run-time group size cost integer divisions per layer (measured 2.9K
// cycles per 128 x 128 layer, 1.15K of them before the sums; profiles/r04_res_timeline.json).
// AS: each layer's activation kind packed the same way (the shipped model: Elu, Elu,
// Elu, none = 0x0111), or 0xFFFFFFFF: read at run time.
template <int NT, int LMAX, int FMAX, bool CTL, unsigned FS = 0x4444u, unsigned GS = 0u, unsigned AS = 0xFFFFFFFFu>
__global__ __launch_bounds__(NT) void policy_resident1_kernel(const DevProgram *__restrict__ Pd,
                                                                      const u64 *req, u64 *actg, unsigned *err,
                                                                      unsigned *done, u64 idle_ticks,
                                                                      const unsigned *yield, DevCtl C) {
  const DevProgram &P = *Pd;
  extern __shared__ float4 lds4[];
  const int S = P.lds_stride;
  float *x0 = reinterpret_cast<float *>(lds4);           // [8][S] layer 0's input rows (zero past in_dim)
  float *xa = x0 + GO2PI_SMALL_MAXB * S;                 // [8][S] hidden layers' rows (ping-pong)
  float *xb = xa + GO2PI_SMALL_MAXB * S;                 // [8][S]
  int *st = reinterpret_cast<int *>(xb + GO2PI_SMALL_MAXB * S);  // [0] leave, [1] epoch, [2] batch, [3] word
  float *obsv = reinterpret_cast<float *>(st + 4);       // [8][in_dim] the request's observation
  // CTL: the LDS image of the tick's inputs (16-byte aligned: q0 is double), then the request rows
  float *cbase = obsv + (GO2PI_SMALL_MAXB * P.in_dim + 3) / 4 * 4;
  const CtlLds CL = ctl_lds(cbase, GO2PI_SMALL_MAXB, P.in_dim);
  float *craw = cbase + ctl_lds_floats(GO2PI_SMALL_MAXB, P.in_dim);  // [B][GO2PI_CTL_RAW + in_dim]
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = 0;  // (RES_STAMP's workgroup index)
  (void)g;
  const int nl = P.nl, in_dim = P.in_dim, nout = P.out_dim;
  // this lane's weight float4s of every layer (and, on a group's lane 0, the bias of
  // its output), in registers for the kernel's life; the layers' other fields are
  // re-read from the program (scalar cache) per request
  float4 w[LMAX][FMAX];
  float bias[LMAX];
#pragma unroll
  for (int l = 0; l < LMAX; ++l) {
    bias[l] = 0.f;
#pragma unroll
    for (int f = 0; f < FMAX; ++f) w[l][f] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (l < nl && l < LMAX) {
      const DevLayer &L = P.L[l];
      const bool lastl = l == nl - 1;
      const int G = r1_group(L.N_pad, lastl ? NT - 64 : NT);
      const int t = lastl ? tid - 64 : tid;  // the final layer skips wave 0 (the poller)
      const int n = t / G, sl = t % G;
      if (t >= 0 && n < L.N_pad) {
        const int T = L.N_pad >> 4;
        const float4 *W = reinterpret_cast<const float4 *>(L.w);
#pragma unroll
        for (int f = 0; f < FMAX; ++f) {
          const int k = 4 * (sl + G * f);
          if (f < (int)((FS >> (4 * l)) & 15u) && k < L.K_pad)
            w[l][f] = W[((size_t)(k >> 4) * T + (n >> 4)) * 64 + (n & 15) + 16 * ((k & 15) >> 2)];
        }
        if (sl == 0) bias[l] = L.bias[n];
      }
    }
  }
  // every program field a request reads, in registers for the kernel's life: after an
  // idle wait the scalar cache has lost the program's lines, and each dependent reload
  // (layer dims -> group size -> addresses; activation kind; the epilogue) is an L2
  // round trip on the request's path. The empty asm makes each value opaque, so the
  // compiler keeps it (in an SGPR, or a VGPR lane when it spills) instead of reloading.
  int lK[LMAX], lNp[LMAX], lact[LMAX], lgr[LMAX];
  float lal[LMAX], lbe[LMAX];
#pragma unroll
  for (int l = 0; l < LMAX; ++l) {
    const DevLayer &L = P.L[l < nl ? l : 0];
    lK[l] = r1_keep(L.K_pad);
    lNp[l] = r1_keep(L.N_pad);
    lgr[l] = GS ? 0 : r1_keep(__builtin_ctz(r1_group(L.N_pad, l == nl - 1 ? NT - 64 : NT)));
    lact[l] = r1_keep(L.act);
    lal[l] = r1_keep(L.alpha);
    lbe[l] = r1_keep(L.beta);
  }
  const int pro_plain = r1_keep((int)(!P.pre_sub && !P.pre_div && !P.pre_mul && !P.pre_clip));
  const int post_tanh = r1_keep(P.post_tanh);
  const float clo = r1_keep(P.clip_lo), chi = r1_keep(P.clip_hi), pscale = r1_keep(P.scale);
  auto post = [&](float v) {
    if (post_tanh) v = tanhf(v);
    return clip_nan(v, clo, chi) * pscale;
  };
  // layer 0's input rows start (and, past in_dim, stay) zero
  for (int i = tid; i < GO2PI_SMALL_MAXB * S; i += NT) x0[i] = 0.f;
  // a one-row act() request with no prologue lands in x0 straight from the poll
  const bool direct = !CTL && pro_plain && 1 + in_dim <= 64 * RES_POLL;
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): the weights are in registers before the first wait
  const unsigned y0 = yield ? __hip_atomic_load(const_cast<unsigned *>(yield), __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT)
                            : 0u;
  unsigned last = 0, nreq = 0;
  (void)nreq;
  for (;;) {
    if (wave == 0) {
      int leave = 0, B = 0;
      unsigned e = 0, word = 0;
      if constexpr (CTL)
        wait_request<__HIP_MEMORY_SCOPE_SYSTEM, 3>(req, GO2PI_CTL_RAW + in_dim, last, idle_ticks, craw, err, lane,
                                                   leave, e, B, word, yield, y0);
      else
        wait_request<__HIP_MEMORY_SCOPE_SYSTEM>(req, in_dim, last, idle_ticks, obsv, err, lane, leave, e, B, word,
                                                yield, y0, direct ? x0 : nullptr);
      RES_STAMP(0);
      RES_CLOCK(15);
      if (lane == 0) {
        st[0] = leave;
        st[1] = (int)e;
        st[2] = B;
        st[3] = (int)word;
      }
    }
    lds_barrier();
    if (st[0]) break;
    const unsigned e = (unsigned)st[1];
    const int B = st[2];
    const unsigned word = (unsigned)st[3];
    (void)word;
    last = e;
    CtlView cv{};
    if constexpr (CTL) {
      // the request's rows (craw: state | joystick | previous obs | previous action, each B
      // rows) into the assembly's LDS image, then the observation assembled into obsv
      const bool joy = (word & GO2PI_RES_JOY) != 0u;
      const int o_jy = B * GO2PI_CTL_STATE_DIM, o_obs = o_jy + B * GO2PI_CTL_JOY_DIM, o_act = o_obs + B * in_dim;
      for (int i = tid; i < o_jy; i += NT) CL.st[i] = craw[i];
      for (int i = tid; i < B * GO2PI_CTL_JOY_DIM; i += NT) CL.jy[i] = craw[o_jy + i];
      for (int i = tid; i < B * in_dim; i += NT) CL.obs[i] = craw[o_obs + i];
      for (int i = tid; i < B * GO2PI_CTL_DOF; i += NT) CL.act[i] = craw[o_act + i];
      if (tid < GO2PI_CTL_DOF) CL.q0[tid] = C.prm->q0[tid];
      if (tid < GO2PI_TILE_ROWS) CL.nanf[tid] = 0u;
      __syncthreads();
      ctl_assemble_flat<false, 2>(P, CL, ctl_q(P, C), joy, B, obsv, in_dim, nullptr, tid, NT);
      DevCtl c = C;
      if (!joy) c.joy = nullptr;
      if (!(word & GO2PI_RES_QDES)) c.q_des = nullptr;
      if (!(word & GO2PI_RES_KP)) c.kp = nullptr;
      if (!(word & GO2PI_RES_KD)) c.kd = nullptr;
      cv = ctl_view(c, CL, 0);
      lds_barrier();
    }
    // layer 0's input rows: the observation through the prologue (x0 past in_dim stays zero),
    // unless the poll wrote the one row there itself
    if (!(direct && B == 1)) {
      if (tid < in_dim)
        for (int b = 0; b < B; ++b) {
          const float v = obsv[b * in_dim + tid];
          x0[b * S + tid] = pro_plain ? v : prologue(P, v, tid);
        }
      lds_barrier();
    }
    RES_STAMP(1);
    RES_CLOCK(13);
    float *X = x0, *Y = xa;
#pragma unroll
    for (int l = 0; l < LMAX; ++l) {
      if (l < nl) {
        const bool lastl = l == nl - 1;
        const int lg = GS ? (int)((GS >> (4 * l)) & 15u) : lgr[l], G = 1 << lg, K = lK[l];
        const int t = lastl ? tid - 64 : tid;
        const int n = t >> lg, sl = t & (G - 1);
        const bool mine = t >= 0 && n < lNp[l];
        const bool kfull = GS != 0u && 4 * G * (int)((FS >> (4 * l)) & 15u) <= K;  // no k past K_pad
        for (int b = 0; b < B; ++b) {
          // two packed (v_pk_fma_f32) chains over the lane's float4s: f even / odd
          f32x2 a0 = {0.f, 0.f}, a1 = {0.f, 0.f};
          if (mine) {
            const float *xr = X + b * S + 4 * sl;
#pragma unroll
            for (int f = 0; f < FMAX; ++f) {
              if (f < (int)((FS >> (4 * l)) & 15u) && (kfull || 4 * (sl + G * f) < K)) {
                const float4 x = *reinterpret_cast<const float4 *>(xr + 4 * G * f);
                f32x2 &a = (f & 1) ? a1 : a0;
                a = __builtin_elementwise_fma(f32x2{x.x, x.y}, f32x2{w[l][f].x, w[l][f].y}, a);
                a = __builtin_elementwise_fma(f32x2{x.z, x.w}, f32x2{w[l][f].z, w[l][f].w}, a);
              }
            }
          }
          if (l < 3 && b == 0) RES_CLOCK(16 + 3 * l);  // layer l: fma chains done (shader clock)
          // (lanes past the layer's outputs, and the final layer's wave 0, join the
          // group sums with zeros: the DPP tree runs on whole rows)
          const float v = r1_group_sum((a0.x + a0.y) + (a1.x + a1.y), G);
          if (l < 3 && b == 0) RES_CLOCK(17 + 3 * l);  // group sums done
          if (mine && sl == 0) {
            // (AS: the kind is a constant once the layer loop is unrolled, and the switch folds)
            const int A = AS != 0xFFFFFFFFu ? (int)((AS >> (4 * l)) & 15u) : lact[l];
            const float y = act_fn(A, lal[l], lbe[l], v + bias[l]);
            if (!lastl) Y[b * S + n] = y;
            else if (n < nout) {
              if constexpr (CTL)
                ctl_store(cv, b, n, post(y));
              else
                __hip_atomic_store(actg + (size_t)b * nout + n, ((u64)e << 32) | __float_as_uint(post(y)),
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
          }
        }
        if (l < 3) RES_CLOCK(18 + 3 * l);  // layer l's outputs stored (this wave's)
        if (!lastl) {
          lds_barrier();
          if (l < 6) RES_STAMP(2 + l);  // layer l's outputs in LDS
          if (l < 3) RES_CLOCK(25 + l);  // (shader clock) past the layer's barrier
          X = Y;
          Y = Y == xa ? xb : xa;
        }
      }
    }
    RES_STAMP(8);  // answer issued (this wave's)
    RES_CLOCK(14);
    if constexpr (CTL) {  // the new observation rows and NaN flags, then the done word
      for (int i = tid; i < B * in_dim; i += NT) C.obs[i] = obsv[i];
      if ((word & GO2PI_RES_STATUS) && tid < B) C.status[tid] = CL.nanf[tid];
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0) __hip_atomic_store(done, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    ++nreq;
  }
  // every wave's answer stores drained before the LEAVE done word (the final layer's
  // granules come from waves 1..15)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) __hip_atomic_store(done, GO2PI_RES_LEAVE, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// ---------------------------------------------------------------------------
// policy_act1_kernel — the one-workgroup resident act() of r05.
// policy_resident1_kernel above gives every output its own group of 8 lanes: a
// 128 x 128 layer then moves 1024 lanes x 64 B of its input row out of LDS (64 KB,
// 256 LDS cycles at 256 B/clk) for 16K MACs, and 16 waves on 4 SIMDs serialise the
// DPP trees: ~1.4K cycles per layer against ~130 of fma issue
// (profiles/r04_res_timeline.json). Here:
//
//  * a dedicated polling wave (wave 0) and A1_CW = 8 compute waves (2 per SIMD);
//  * a wide layer (N_pad = H, 64 or 128 outputs) gives each 16-lane DPP row R = H/32
//    outputs: lane s of row g holds the weight float4s k = 64 f + 4 s .. +3 of the
//    outputs 4g + r (R = 4), so one broadcast ds_read_b128 of the input feeds R
//    output chains: 16 KB of LDS reads per 128 x 128 layer, a quarter of r04's;
//  * the R partials are summed by a reduce-scatter over the row (row_ror:8, then
//    row_half_mirror, then quad xor 2 and xor 1: five DPP adds for R = 4, no select),
//    because lane s keeps its outputs in a rotated register order (a1_out);
//  * the final layer (16 outputs, the head) runs on the first four compute waves,
//    one output per DPP row, and its rows' first lanes store the answer granules;
//  * the polling wave keeps D sweeps of the request granules in flight at once
//    (a new sweep issued before the oldest is checked), so a request lands within
//    one PCIe read round trip plus RTT / D instead of plus up to a whole RTT; it
//    takes no part in the arithmetic, so its in-flight poll loads never sit in
//    front of a compute wave's wait.
// Summation order per output: two packed fma chains per register (x.xy, x.zw)
// over the lane's float4s, their sum, then the fixed DPP tree: deterministic,
// within the 1e-5 contract of the fp64 oracle (not the MFMA path's order).

// A1_STAMP: RESCLK diagnostics, wall clock (slot i) / shader clock (A1_CLOCK) of the
// first compute lane (tid 64) or, for the poll marks, of the polling wave (tid 0).
#ifdef GO2PI_DIAG_RESCLK
// (global stores, not flat: a flat store counts in lgkmcnt too, and every LDS wait after
// a stamp waited for the stamp's L2 write)
#define A1_STAMP(t, i)                                                                             \
  do {                                                                                             \
    if (P.stamps && tid == (t))                                                                    \
      ((gu64_t *)P.stamps)[(size_t)(nreq & 511) * 32 + (i)] = wall_clock64();                      \
  } while (0)
#define A1_CLOCK(t, i)                                                                             \
  do {                                                                                             \
    if (P.stamps && tid == (t))                                                                    \
      ((gu64_t *)P.stamps)[(size_t)(nreq & 511) * 32 + (i)] = __builtin_amdgcn_s_memtime();        \
  } while (0)
#else
#define A1_STAMP(t, i) \
  do {                 \
  } while (0)
#define A1_CLOCK(t, i) \
  do {                 \
  } while (0)
#endif

// NL: dense layers (2..4): NL - 1 wide layers of H outputs (H = 64 or 128), then the
// 16-output head. F0: layer 0's float4s per lane (K0_pad <= 64 F0). AS: the layers'
// activation kinds, 4 bits each (layer l at 4l; the shipped model: 0x0111), or
// 0xFFFFFFFF: read at run time. D: poll sweeps in flight. PRO: the program has an
// observation prologue (Sub / Div / Mul / Clip), applied by the polling wave. CW:
// compute waves, 8 (two per SIMD, R = H / 32 outputs per lane) or 4 (one per SIMD,
// R = H / 16: twice the weights per lane, half the lanes' reduction overhead).
// CTL: the controller tick (go2pi_controller_step at batch <= 8; launch_resident's ctl
// semantics): the request carries the tick's raw rows, which the polling wave puts
// straight into the assembly's LDS image; the compute waves assemble the observation
// (ctl_fn.hpp, the code of the batched kernel: the new rows go to the host staging, the
// normalised ones to x0), run the layers, post-process the action into the staging
// (ctl_store) and set the done word behind every output's drain.
template <int NL, int H, int F0, unsigned AS, int D, bool PRO, int CW = 8, bool CTL = false>
__global__ __launch_bounds__(a1_nt(CW)) void policy_act1_kernel(const DevProgram *__restrict__ Pd, const u64 *req,
                                                                u64 *actg, unsigned *err, unsigned *done,
                                                                u64 idle_ticks, const unsigned *yield, DevCtl C) {
  static_assert(NL >= 2 && NL <= 4 && (H == 64 || H == 128) && F0 >= 1 && F0 <= 4 && (CW == 4 || CW == 8),
                "policy_act1_kernel shape");
  constexpr int NT = a1_nt(CW);
  constexpr int R = H / (4 * CW);  // outputs per lane in a wide layer (a DPP row of 16 lanes: 16 R / 16)
  constexpr int HF = H / 64;  // float4s per lane of a K = H layer
  constexpr int NM = NL - 2 > 0 ? NL - 2 : 1;  // wide layers after layer 0 (array extent)
  constexpr int NP = CTL ? 3 : A1_NP;          // granule loads per lane per sweep
  // CTL: layer 0's and the head's weights live in LDS, not registers (re-read per request,
  // 8 + 2 ds_read_b128 per lane for the shipped model): beside the assembly's registers
  // they spilled
  constexpr bool W0L = CTL;
  const DevProgram &P = *Pd;
  extern __shared__ float4 lds4[];
  const int S = P.lds_stride;
  float *x0 = reinterpret_cast<float *>(lds4);  // [8][S] layer 0's input rows (zero past in_dim)
  float *xa = x0 + GO2PI_SMALL_MAXB * S;        // [8][S] wide layers' rows (ping-pong)
  float *xb = xa + GO2PI_SMALL_MAXB * S;
  int *st = reinterpret_cast<int *>(xb + GO2PI_SMALL_MAXB * S);  // [0] leave, [1] epoch, [2] batch, [3] word
  // CTL: the LDS image of the tick's inputs (q0 once, the request's rows per request),
  // then layer 0's weights, lane-major [f][j][compute lane] float4 (a wave's read: 1 KiB
  // contiguous)
  const CtlLds CL = ctl_lds(reinterpret_cast<float *>(st + 4), GO2PI_SMALL_MAXB, P.in_dim);
  float4 *w0l = reinterpret_cast<float4 *>(reinterpret_cast<float *>(st + 4) +
                                           (CTL ? ctl_lds_floats(GO2PI_SMALL_MAXB, P.in_dim) : 0));
  // CTL: the head's weights too (lane-major [f][head lane], 256 lanes), then the request's
  // new observation rows [B][in_dim]
  float4 *wol = w0l + (W0L ? F0 * R * 64 * CW : 0);
  float *obsn = reinterpret_cast<float *>(wol + (W0L ? HF * 256 : 0));
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int c = tid - 64;                // compute lane (the polling wave: negative)
  const int s = c & 15, grp = c >> 4;    // k-slice within the DPP row, the row
  const int in_dim = P.in_dim, nout = P.out_dim;
  // ---- weights in registers for the kernel's life (zero where k >= K_pad)
  float4 w0[F0][R], wm[NM][HF][R], wo[HF];
  float bw[NL - 1], bo = 0.f;
  auto wld = [&](const DevLayer &L, int n, int k) {
    const int T = L.N_pad >> 4;
    const float4 *W = reinterpret_cast<const float4 *>(L.w);
    return k < L.K_pad ? W[((size_t)(k >> 4) * T + (n >> 4)) * 64 + (n & 15) + 16 * ((k & 15) >> 2)]
                       : make_float4(0.f, 0.f, 0.f, 0.f);
  };
  const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int l = 0; l < NL - 1; ++l) {
    bw[l] = 0.f;
    const DevLayer &L = P.L[l];
#pragma unroll
    for (int j = 0; j < R; ++j) {
      const int n = R * grp + a1_out<R>(j, s);
      if (l == 0) {
#pragma unroll
        for (int f = 0; f < F0; ++f) w0[f][j] = c >= 0 ? wld(L, n, 64 * f + 4 * s) : z4;
      } else {
#pragma unroll
        for (int f = 0; f < HF; ++f) wm[l - 1][f][j] = c >= 0 ? wld(L, n, 64 * f + 4 * s) : z4;
      }
    }
    if (c >= 0) bw[l] = L.bias[R * grp + a1_fin<R>(s)];
  }
  if constexpr (NL == 2) {
#pragma unroll
    for (int f = 0; f < HF; ++f)
#pragma unroll
      for (int j = 0; j < R; ++j) wm[0][f][j] = z4;
  }
  {
    const DevLayer &L = P.L[NL - 1];
    const bool hl = c >= 0 && c < 256;
#pragma unroll
    for (int f = 0; f < HF; ++f) wo[f] = hl ? wld(L, grp, 64 * f + 4 * s) : z4;
    if (hl) bo = L.bias[grp];
  }
  // the program fields a request reads, in SGPRs for the kernel's life (run-time
  // activations). With the activations compiled in (AS) the launcher has checked the
  // hidden layers' Elu alpha is 1 and the head has none, and the post-processing
  // fields are left to the compiler: pinned in SGPRs beside the controller form's
  // parameters they spilled 63 SGPRs into VGPR lanes, and those to scratch.
  constexpr bool ACT_RT = AS == 0xFFFFFFFFu;
  int lact[NL];
  float lal[NL], lbe[NL];
#pragma unroll
  for (int l = 0; l < NL; ++l) {
    lact[l] = ACT_RT ? r1_keep(P.L[l].act) : 0;
    lal[l] = ACT_RT ? r1_keep(P.L[l].alpha) : 1.f;
    lbe[l] = ACT_RT ? r1_keep(P.L[l].beta) : 0.f;
  }
  const int post_tanh = ACT_RT ? r1_keep(P.post_tanh) : P.post_tanh;
  const float clo = ACT_RT ? r1_keep(P.clip_lo) : P.clip_lo, chi = ACT_RT ? r1_keep(P.clip_hi) : P.clip_hi;
  const float pscale = ACT_RT ? r1_keep(P.scale) : P.scale;
  // the polling wave: each lane's prologue constants for its granule positions (the
  // column of granule i is (i - 1) mod in_dim whatever the batch)
  const Pro pro = PRO ? pro_of(P) : Pro{};
  ProK pk[NP];
#pragma unroll
  for (int u = 0; u < NP; ++u) {
    const int i = u * 64 + lane;
    pk[u] = (PRO && wave == 0 && i >= 1) ? pro_k(pro, (i - 1) % in_dim) : ProK{0.f, 1.f, 1.f};
  }
  for (int i = tid; i < GO2PI_SMALL_MAXB * S; i += NT) x0[i] = 0.f;
  if constexpr (W0L) {
    if (c >= 0)
#pragma unroll
      for (int f = 0; f < F0; ++f)
#pragma unroll
        for (int j = 0; j < R; ++j) w0l[(f * R + j) * 64 * CW + c] = w0[f][j];
    if (c >= 0 && c < 256)
#pragma unroll
      for (int f = 0; f < HF; ++f) wol[f * 256 + c] = wo[f];
  }
  if constexpr (CTL) {
    if (tid < 2 * GO2PI_CTL_DOF) reinterpret_cast<float *>(CL.q0)[tid] = reinterpret_cast<const float *>(C.prm->q0)[tid];
    if (tid < GO2PI_TILE_ROWS) CL.nanf[tid] = 0u;
  }
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): weights and constants in registers before the first wait
  const unsigned y0 = __hip_atomic_load(const_cast<unsigned *>(yield), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();  // x0 cleared before the poller writes a row into it
  unsigned last = 0, nreq = 0;
  (void)nreq;
  u64 pv[D][NP];  // the polling wave's sweep registers (a1_poll)
  unsigned pyv[D];
#pragma unroll
  for (int d = 0; d < D; ++d) {
    pyv[d] = 0u;
#pragma unroll
    for (int u = 0; u < NP; ++u) pv[d][u] = 0ull;
  }
  const int per = CTL ? GO2PI_CTL_RAW + in_dim : in_dim;  // request floats per robot
  for (;;) {
    if (wave == 0) {
      unsigned e = 0, word = 0;
      int B = 1;
      int got;
      if constexpr (CTL) {
        got = a1_poll<D, NP>(req, per, last, idle_ticks, err, lane, e, B, word, yield, y0, pv, pyv,
                             [&](int, int i, float x) { a1_put_ctl(CL, in_dim, B, i, x); },
                             [&](int i, float x) { a1_put_ctl(CL, in_dim, B, i, x); });
      } else {
        got = a1_poll<D, NP>(
            req, per, last, idle_ticks, err, lane, e, B, word, yield, y0, pv, pyv,
            [&](int u, int i, float x) { a1_put(x0, S, in_dim, B, i, PRO ? prologue(pro, pk[u], x) : x); },
            [&](int i, float x) { a1_put(x0, S, in_dim, B, i, PRO ? prologue(pro, x, (i - 1) % in_dim) : x); });
      }
      A1_STAMP(0, 0);
      A1_CLOCK(0, 15);
      if (lane == 0) {
        st[0] = !got;
        st[1] = (int)e;
        st[2] = B;
        st[3] = (int)word;
      }
    }
    lds_barrier();  // the request's rows are in x0 (CTL: in the assembly's image)
    // (row 0's layer-0 input read beside the request word: one LDS round trip, not two)
    float4 xpre[F0];
#pragma unroll
    for (int f = 0; f < F0; ++f) xpre[f] = *reinterpret_cast<const float4 *>(x0 + 64 * f + 4 * s);
    const int4 sv = *reinterpret_cast<const int4 *>(st);
    if (sv.x) break;
    const unsigned e = (unsigned)sv.y;
    const int B = sv.z;
    const unsigned word = (unsigned)sv.w;
    last = e;
    if (wave == 0) {  // the poller passes the request's barriers, then polls again
#pragma unroll
      for (int l = 0; l + 1 < NL; ++l) lds_barrier();
      if constexpr (CTL) {
        lds_barrier();  // the assembly
        lds_barrier();  // the outputs drained (the done word)
      }
      ++nreq;
      continue;
    }
    if constexpr (CTL) {
      A1_STAMP(64, 10);
      // the observation assembled from the image: the new rows to LDS (obsn; they go to the
      // host staging with the other outputs after the head), their normalised values to x0
      // (the padding rows past B, which it zero-fills, reach into xa: written by layer 0
      // before any read). Stored straight to the host staging here, the rows' PCIe stores
      // sat in front of every later wait of the request.
      A1_CLOCK(64, 11);
      const bool joy = (word & GO2PI_RES_JOY) != 0u;
      const CtlQ q = ctl_q(P, C);
#ifdef GO2PI_DIAG_RESCLK
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // (the parameters' arrival timed on its own)
#endif
      A1_CLOCK(64, 19);
      // (ctl_assemble_flat's two passes, timed apart: shader-clock slots 19-21)
      // (x0's padding columns stay zero from the start and its rows past B are never read:
      // the shift pass leaves them alone)
      static_assert(CW >= 7, "the controller form's assembly runs one history block per compute wave");
      // the shift pass starts on the last compute wave, the one without a block (at batch 1
      // its elements all fit that wave: the two passes run side by side)
      const int cr = c + 64 < 64 * CW ? c + 64 : c + 64 - 64 * CW;
      if (q.pro.sub || q.pro.div || q.pro.mul) {
        ctl_append_waves<true, true>(CL, q, joy, B, x0, S, obsn, c);
        A1_CLOCK(64, 20);
        ctl_shift<true, true, 2, false>(CL, q, B, x0, S, obsn, cr, 64 * CW);
      } else {
        ctl_append_waves<true, false>(CL, q, joy, B, x0, S, obsn, c);
        A1_CLOCK(64, 20);
        ctl_shift<true, false, 2, false>(CL, q, B, x0, S, obsn, cr, 64 * CW);
      }
      A1_CLOCK(64, 21);
#ifdef GO2PI_DIAG_ASM2  // both passes again, warm (instruction fetch and first touches vs. work): slots 22-23
      ctl_append_waves<true, false>(CL, q, joy, B, x0, S, obsn, c);
      A1_CLOCK(64, 22);
      ctl_shift<true, false, 2, false>(CL, q, B, x0, S, obsn, cr, 64 * CW);
      A1_CLOCK(64, 23);
#endif
      lds_barrier();
#pragma unroll
      for (int f = 0; f < F0; ++f) xpre[f] = *reinterpret_cast<const float4 *>(x0 + 64 * f + 4 * s);
      // the new observation rows and NaN flags answer now, their stores overlapping the layers
      const CtlGran G = ctl_gran(in_dim);
      for (int i = c; i < B * in_dim; i += 64 * CW) {
        int ii = i;
        asm volatile("" : "+v"(ii));  // (the addresses formed here, not hoisted and spilled)
        gran_put(actg + G.obs + ii, e, __float_as_uint(obsn[ii]));
      }
      if ((word & GO2PI_RES_STATUS) && c < B) {
        int cs = c;
        asm volatile("" : "+v"(cs));
        gran_put(actg + G.status + cs, e, CL.nanf[cs]);
      }
    }
    A1_STAMP(64, 1);
    A1_CLOCK(64, 13);
    // ---- wide layers
    float *X = x0, *Y = xa;
#pragma unroll
    for (int l = 0; l < NL - 1; ++l) {
      const int A = AS != 0xFFFFFFFFu ? (int)((AS >> (4 * l)) & 15u) : lact[l];
      for (int b = 0; b < B; ++b) {
        f32x2 acc[R];
#pragma unroll
        for (int j = 0; j < R; ++j) acc[j] = f32x2{0.f, 0.f};
        const float *xr = X + b * S + 4 * s;
        if (l == 0) {
#pragma unroll
          for (int f = 0; f < F0; ++f) {
            const float4 x = b == 0 ? xpre[f] : *reinterpret_cast<const float4 *>(xr + 64 * f);
#pragma unroll
            for (int j = 0; j < R; ++j) {
              const float4 wv = W0L ? w0l[(f * R + j) * 64 * CW + c] : w0[f][j];
              acc[j] = __builtin_elementwise_fma(f32x2{x.x, x.y}, f32x2{wv.x, wv.y}, acc[j]);
              acc[j] = __builtin_elementwise_fma(f32x2{x.z, x.w}, f32x2{wv.z, wv.w}, acc[j]);
            }
          }
        } else {
#pragma unroll
          for (int f = 0; f < HF; ++f) {
            const float4 x = *reinterpret_cast<const float4 *>(xr + 64 * f);
#pragma unroll
            for (int j = 0; j < R; ++j) {
              const float4 wv = wm[l > 0 ? l - 1 : 0][f][j];
              acc[j] = __builtin_elementwise_fma(f32x2{x.x, x.y}, f32x2{wv.x, wv.y}, acc[j]);
              acc[j] = __builtin_elementwise_fma(f32x2{x.z, x.w}, f32x2{wv.z, wv.w}, acc[j]);
            }
          }
        }
        if (l == 0 && b == 0) A1_CLOCK(64, 16);
        float p[R];
#pragma unroll
        for (int j = 0; j < R; ++j) p[j] = acc[j].x + acc[j].y;
        const float v = a1_reduce<R>(p);
        if (l == 0 && b == 0) A1_CLOCK(64, 17);
        if ((s & (16 / R - 1)) == 0) Y[b * S + R * grp + a1_fin<R>(s)] = act_fn(A, lal[l], lbe[l], v + bw[l]);
      }
      if (l == 0) A1_CLOCK(64, 18);
      lds_barrier();
      if (l < 6) A1_STAMP(64, 2 + l);
      if (l < 3) A1_CLOCK(64, 25 + l);
      X = Y;
      Y = Y == xa ? xb : xa;
    }
    // ---- the head: 16 outputs, one per DPP row of compute waves 0..3
    if (c < 256) {
      const int A = AS != 0xFFFFFFFFu ? (int)((AS >> (4 * (NL - 1))) & 15u) : lact[NL - 1];
      for (int b = 0; b < B; ++b) {
        f32x2 acc = {0.f, 0.f};
        const float *xr = X + b * S + 4 * s;
#pragma unroll
        for (int f = 0; f < HF; ++f) {
          const float4 x = *reinterpret_cast<const float4 *>(xr + 64 * f);
          const float4 wv = W0L ? wol[f * 256 + c] : wo[f];
          acc = __builtin_elementwise_fma(f32x2{x.x, x.y}, f32x2{wv.x, wv.y}, acc);
          acc = __builtin_elementwise_fma(f32x2{x.z, x.w}, f32x2{wv.z, wv.w}, acc);
        }
        float p[1] = {acc.x + acc.y};
        const float v = a1_reduce<1>(p);
        if (s == 0 && grp < nout) {
          float y = act_fn(A, lal[NL - 1], lbe[NL - 1], v + bo);
          if (post_tanh) y = tanhf(y);
          y = clip_nan(y, clo, chi) * pscale;
          if constexpr (CTL) {
            Y[b * 16 + grp] = y;  // (the answer granules from there: below)
          } else {
            int n = grp;
            asm volatile("" : "+v"(n));  // (the granule address formed here, not hoisted and spilled)
            __hip_atomic_store(actg + (size_t)b * nout + n, ((u64)e << 32) | __float_as_uint(y), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
          }
        }
      }
    }
    A1_STAMP(64, 8);
    A1_CLOCK(64, 14);
    if constexpr (CTL) {
      // The answer's action, q_des, kp and kd granules, written by consecutive threads from
      // the head's outputs gathered in LDS (Y: not the head's input), so that each store
      // instruction covers one contiguous range of the host's staging: stored by the head's
      // lanes themselves (four per wave, each output's granules apart) the partial-line
      // PCIe writes cost ~6 us per tick. The image's joystick and q0 rows stay valid: the
      // polling wave stages the next request only after the host has read this answer.
      lds_barrier();
      if (c < GO2PI_TILE_ROWS) CL.nanf[c] = 0u;  // (the status granule read it after the assembly)
      if (c < B * GO2PI_CTL_DOF) {
        DevCtl cc = C;
        if (!(word & GO2PI_RES_JOY)) cc.joy = nullptr;
        if (!(word & GO2PI_RES_QDES)) cc.q_des = nullptr;
        if (!(word & GO2PI_RES_KP)) cc.kp = nullptr;
        if (!(word & GO2PI_RES_KD)) cc.kd = nullptr;
        const CtlView cv = ctl_view(cc, CL, 0);
        int i = c;
        asm volatile("" : "+v"(i));  // (the addresses formed here, not hoisted and spilled)
        const int b = i / GO2PI_CTL_DOF, n = i - b * GO2PI_CTL_DOF;
        ctl_store_gran(cv, b, n, Y[b * 16 + n], actg, ctl_gran(in_dim), e);
      }
      A1_STAMP(64, 9);
    }
    ++nreq;
  }
  // leaving: every wave's answer stores (and the poller's sweeps) drained before the
  // LEAVE done word, so a host that sees LEAVE and rescans finds a served request's
  // granules (engine.cpp resident_serve)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) __hip_atomic_store(done, GO2PI_RES_LEAVE, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}


// The generic act1 instantiations, by shape (AS run time, PRO, CW = 8; two sweeps in
// flight, one where the weights leave no room for the second: act1_fits).
template <int NL, int H, class GO>
int a1_generic_f0(int f0, GO &go1) {
  constexpr int D2 = (H == 128 && NL == 4) ? 1 : 2, D4 = (H == 128 && NL == 3) ? 1 : 2;
  if (f0 == 1) return go1(policy_act1_kernel<NL, H, 1, 0xFFFFFFFFu, 2, true, 8>, 8);
  if (f0 == 2) return go1(policy_act1_kernel<NL, H, 2, 0xFFFFFFFFu, D2, true, 8>, 8);
  if constexpr (!(H == 128 && NL == 4)) return go1(policy_act1_kernel<NL, H, 4, 0xFFFFFFFFu, D4, true, 8>, 8);
  return (int)hipErrorInvalidValue;  // (act1_shape refuses it)
}
// ... and of the controller form (the assembly applies the prologue: PRO false; D = 1)
template <int NL, int H, class GO>
int a1_generic_ctl_f0(int f0, GO &go1) {
  if (f0 == 1) return go1(policy_act1_kernel<NL, H, 1, 0xFFFFFFFFu, 1, false, 8, true>, 8);
  if (f0 == 2) return go1(policy_act1_kernel<NL, H, 2, 0xFFFFFFFFu, 1, false, 8, true>, 8);
  if constexpr (!(H == 128 && NL == 4)) return go1(policy_act1_kernel<NL, H, 4, 0xFFFFFFFFu, 1, false, 8, true>, 8);
  return (int)hipErrorInvalidValue;  // (act1_shape refuses it)
}
template <class GO>
int a1_generic_ctl(const A1Shape &a, GO &go1) {
  if (a.h == 128) {
    if (a.nl == 2) return a1_generic_ctl_f0<2, 128>(a.f0, go1);
    if (a.nl == 3) return a1_generic_ctl_f0<3, 128>(a.f0, go1);
    return a1_generic_ctl_f0<4, 128>(a.f0, go1);
  }
  if (a.nl == 2) return a1_generic_ctl_f0<2, 64>(a.f0, go1);
  if (a.nl == 3) return a1_generic_ctl_f0<3, 64>(a.f0, go1);
  return a1_generic_ctl_f0<4, 64>(a.f0, go1);
}
template <class GO>
int a1_generic(const A1Shape &a, GO &go1) {
  if (a.h == 128) {
    if (a.nl == 2) return a1_generic_f0<2, 128>(a.f0, go1);
    if (a.nl == 3) return a1_generic_f0<3, 128>(a.f0, go1);
    return a1_generic_f0<4, 128>(a.f0, go1);
  }
  if (a.nl == 2) return a1_generic_f0<2, 64>(a.f0, go1);
  if (a.nl == 3) return a1_generic_f0<3, 64>(a.f0, go1);
  return a1_generic_f0<4, 64>(a.f0, go1);
}
A1Shape act1_shape(const DevProgram &p) {
  A1Shape a{0, 0, 0};
  if (p.has_gru || p.nl < 2 || p.nl > 4 || p.L[p.nl - 1].N_pad != 16) return a;
  const int H = p.L[0].N_pad;
  if (H != 64 && H != 128) return a;
  for (int l = 1; l < p.nl; ++l)
    if (p.L[l].K_pad != H || (l + 1 < p.nl && p.L[l].N_pad != H)) return a;
  int f0 = (p.L[0].K_pad + 63) / 64;
  if (f0 == 3) f0 = 4;
  // (layer 0's lanes read their input row up to 64 F0: inside the row, zero past in_dim)
  if (f0 > 4 || p.lds_stride < std::max(64 * f0, H)) return a;
  // weights per lane beyond the registers of 3 waves per SIMD (168): the r04 form
  if (H == 128 && p.nl == 4 && f0 == 4) return a;
  a.nl = p.nl;
  a.h = H;
  a.f0 = f0;
  return a;
}

size_t resident1_lds_bytes(const DevProgram &p, bool ctl) {
  size_t f = 3 * (size_t)GO2PI_SMALL_MAXB * p.lds_stride + 4 + ((size_t)GO2PI_SMALL_MAXB * p.in_dim + 3) / 4 * 4;
  if (ctl) f += (size_t)ctl_lds_floats(GO2PI_SMALL_MAXB, p.in_dim) + (size_t)GO2PI_SMALL_MAXB * (GO2PI_CTL_RAW + p.in_dim);
  return sizeof(float) * f;
}

int launch_resident1(const DevProgram &p, const DevProgram *p_dev, const unsigned long long *req,
                     unsigned long long *actg, unsigned *err, unsigned *done, unsigned long long idle_ticks,
                     const unsigned *yield, const DevCtl *ctl, void *stream) {
  if (!resident1_fits(p, ctl != nullptr)) return (int)hipErrorInvalidValue;
  const size_t lds = resident1_lds_bytes(p, ctl != nullptr);  // (r04's forms)
  auto go = [&](auto kern, int nt) {
    if (lds > 160 * 1024) return (int)hipErrorInvalidValue;
    if (lds > 64 * 1024) {
      const hipError_t a = hipFuncSetAttribute(reinterpret_cast<const void *>(kern),
                                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      if (a != hipSuccess) return (int)a;
    }
    hipLaunchKernelGGL(kern, dim3(1), dim3(nt), lds, reinterpret_cast<hipStream_t>(stream), p_dev, req, actg,
                       err, done, idle_ticks, yield, ctl ? *ctl : DevCtl{});
    return (int)hipGetLastError();
  };
  // the shipped model's shape (98 -> 128^3 -> 12: 4, 4, 4, 1 float4s per lane) has its own
  // instantiation: the registers it leaves free keep the controller form out of scratch
  // (Elu alpha 1 on the hidden layers, no activation on the head: the exported policy's)
  const bool elu1 = r1_acts(p) == 0x0111u && p.L[0].alpha == 1.f && p.L[1].alpha == 1.f && p.L[2].alpha == 1.f;
  // r05: the polling-wave form (policy_act1_kernel) wherever its shape applies
  // (GO2PI_RES_R1W=1: the r04 1024-thread form, A/B diagnostics; GO2PI_A1_DEPTH: poll
  // sweeps in flight, 1 / 2 / 4)
  const A1Shape a1 = act1_shape(p);
  if (a1.nl && !std::getenv("GO2PI_RES_R1W")) {
    // (the controller form: the assembly's image, layer 0's weights, lane-major, and the
    // new observation rows besides)
    const size_t lds1 = sizeof(float) * (3 * (size_t)GO2PI_SMALL_MAXB * p.lds_stride + 4 +
                                         (ctl ? (size_t)ctl_lds_floats(GO2PI_SMALL_MAXB, p.in_dim) +
                                                    (size_t)a1.f0 * (a1.h / 32) * 512 * 4 + (size_t)(a1.h / 64) * 256 * 4 +
                                                    (size_t)GO2PI_SMALL_MAXB * p.in_dim
                                              : 0));
    auto go1 = [&](auto kern, int cw) {
      if (lds1 > 64 * 1024) {
        const hipError_t a = hipFuncSetAttribute(reinterpret_cast<const void *>(kern),
                                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds1);
        if (a != hipSuccess) return (int)a;
      }
      // (yield never null: the kernel loads it unconditionally, see a1_poll)
      hipLaunchKernelGGL(kern, dim3(1), dim3(a1_nt(cw)), lds1, reinterpret_cast<hipStream_t>(stream), p_dev, req, actg,
                         err, done, idle_ticks, yield ? yield : reinterpret_cast<const unsigned *>(p.zero),
                         ctl ? *ctl : DevCtl{});
      return (int)hipGetLastError();
    };
    const char *dv = std::getenv("GO2PI_A1_DEPTH");
    const int depth = dv ? std::atoi(dv) : 2;
    const bool pro = p.pre_sub || p.pre_div || p.pre_mul || p.pre_clip;
    const char *cv = std::getenv("GO2PI_A1_CW");
    const int cw = cv && std::atoi(cv) == 4 ? 4 : 8;
    if (ctl) {  // the controller form: one sweep in flight (three loads per lane), eight compute waves
      if (a1.nl == 4 && a1.h == 128 && a1.f0 == 2 && elu1)
        return go1(policy_act1_kernel<4, 128, 2, 0x0111u, 1, false, 8, true>, 8);
      return a1_generic_ctl(a1, go1);
    }
    if (a1.nl == 4 && a1.h == 128 && a1.f0 == 2 && elu1 && !pro) {
      if (cw == 8) {
        if (depth == 1) return go1(policy_act1_kernel<4, 128, 2, 0x0111u, 1, false, 8>, 8);
        return go1(policy_act1_kernel<4, 128, 2, 0x0111u, 2, false, 8>, 8);
      }
      if (depth == 1) return go1(policy_act1_kernel<4, 128, 2, 0x0111u, 1, false, 4>, 4);
      return go1(policy_act1_kernel<4, 128, 2, 0x0111u, 2, false, 4>, 4);
    }
    // every other act1 shape: activations and the prologue read at run time, two sweeps
    // in flight, eight compute waves
    return a1_generic(a1, go1);
  }
  if (ctl) {  // r04's forms
    if (p.nl == 4 && elu1 && r1_shape(p, 512) == 0x2887u && r1_lgs(p, 512) == 0x4222u)
      return go(policy_resident1_kernel<512, R1_LMAX, 8, true, 0x2887u, 0x4222u, 0x0111u>, 512);
    return go(policy_resident1_kernel<512, R1_LMAX, 8, true, 0x8888u>, 512);
  }
  if (p.nl == 4 && elu1 && r1_shape(p, 1024) == 0x2444u && r1_lgs(p, 1024) == 0x4333u)
    return go(policy_resident1_kernel<1024, R1_LMAX, 4, false, 0x2444u, 0x4333u, 0x0111u>, 1024);
  return go(policy_resident1_kernel<1024, R1_LMAX, 4, false>, 1024);
}

int launch_resident(const DevProgram &p, const DevProgram *p_dev, const unsigned long long *req,
                    unsigned long long *actg,
                    unsigned long long *gran, int gstride, unsigned long long *mirror, unsigned *err,
                    unsigned *done, unsigned long long idle_ticks, const DevCtl *ctl, unsigned long long *hgran,
                    float *hidden, const unsigned *yield, void *stream) {
  if (p.L[p.nl - 1].N_pad != 16) return (int)hipErrorInvalidValue;  // workgroup 0 owns the whole action
  for (int l = 0; l < p.nl; ++l)
    if (p.L[l].K_pad > RES_MAXS * RES_WAVES * 16) return (int)hipErrorInvalidValue;
  const bool rnn = p.has_gru != 0;
  const bool lstm = rnn && p.gru.cell == 1;
  if (rnn && (ctl || p.gru.cell > 1 || (!lstm && p.gru.lbr != 1) || p.gru.H % 64 ||
              p.gru.I_pad + p.gru.H > RES_GS * RES_WAVES * 16 || !hgran || !hidden))
    return (int)hipErrorInvalidValue;
  // local layer 0 where each thread's share of it fits NF = 8, 12 or 16 registers'
  // fragments (a slice's chunks past layer 0's own are zero fragments on zero columns)
  const int N0 = p.L[0].N_pad, C0 = p.L[0].K_pad >> 4;
  const int KS = (N0 > 0 && (RES_WAVES * 64) % N0 == 0) ? (RES_WAVES * 64) / N0 : 0;
  const int nf = KS > 0 ? 4 * ((C0 + KS - 1) / KS) : 0;
  const bool local0 = !rnn && p.nl >= 2 && (nf == 8 || nf == 12 || nf == 16) && !std::getenv("GO2PI_RES_TILED0");
  const int x0len = local0 ? (nf / 4) * KS * 16 : p.L[0].K_pad;
  // one workgroup per 16-output tile of the widest TILED layer (with a local layer 0,
  // workgroups beyond the later layers' tiles would only repeat layer 0 and poll)
  int grid = rnn ? (p.gru.H >> 4) : 1;
  for (int l = local0 ? 1 : 0; l < p.nl; ++l) grid = std::max(grid, p.L[l].N_pad >> 4);
  // (the kernel's LDS carve-up: x0 and p0 are laid out whether used or not)
  const size_t ctl_off = ((size_t)GO2PI_SMALL_MAXB * p.lds_stride + RES_WAVES * GO2PI_SMALL_MAXB * 16 + 4 +
                          (size_t)GO2PI_SMALL_MAXB * p.in_dim + (size_t)GO2PI_SMALL_MAXB * x0len +
                          (size_t)(KS > 1 ? KS : 0) * GO2PI_SMALL_MAXB * N0 + 3) / 4 * 4;
  size_t tail = 0;
  if (ctl) tail = (size_t)ctl_lds_floats(GO2PI_SMALL_MAXB, p.in_dim) + (size_t)GO2PI_SMALL_MAXB * (GO2PI_CTL_RAW + p.in_dim);
  if (rnn)
    tail = (size_t)GO2PI_SMALL_MAXB * (p.gru.I_pad + p.gru.H) + RES_WAVES * 4 * GO2PI_SMALL_MAXB * 16 +
           2 * GO2PI_SMALL_MAXB + 4 * GO2PI_SMALL_MAXB * 16;  // hown, cown, hst, cst (laid out for a GRU too)
  const size_t lds = sizeof(float) * (ctl_off + tail);
  if (lds > 160 * 1024) return (int)hipErrorInvalidValue;
  auto go = [&](auto kern) {
    if (lds > 64 * 1024) {
      const hipError_t a = hipFuncSetAttribute(reinterpret_cast<const void *>(kern),
                                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      if (a != hipSuccess) return (int)a;
    }
    hipLaunchKernelGGL(kern, dim3(grid), dim3(RES_WAVES * 64), lds, reinterpret_cast<hipStream_t>(stream), p_dev, req,
                       actg, gran, gstride, mirror, err, done, idle_ticks, ctl ? *ctl : DevCtl{}, hgran, hidden, yield);
    return (int)hipGetLastError();
  };
  if (lstm) return go(policy_resident_kernel<0, false, 2>);
  if (rnn) return go(policy_resident_kernel<0, false, 1>);
  if (ctl) {
    if (local0 && nf == 8) return go(policy_resident_kernel<8, true>);
    if (local0 && nf == 12) return go(policy_resident_kernel<12, true>);
    if (local0 && nf == 16) return go(policy_resident_kernel<16, true>);
    return go(policy_resident_kernel<0, true>);
  }
  if (local0 && nf == 8) return go(policy_resident_kernel<8, false>);
  if (local0 && nf == 12) return go(policy_resident_kernel<12, false>);
  if (local0 && nf == 16) return go(policy_resident_kernel<16, false>);
  return go(policy_resident_kernel<0, false>);
}

}  // namespace go2pi
