// policy_wide_kernel — the resident batch <= 8 act() for wide dense policies (r06).
//
// BASELINE configs[1]: the 48 -> 512^3 -> 12 Go2 policy at batch 1, one
// ONNXActor::act() per control tick (onnx_inference/src/cpp/onnx_actor.cpp:38-48,
// timed by main.cpp:38-42). Its weights (2.2 MB) cannot sit in one CU, so the
// request crosses workgroups. The r03 form (policy_resident_kernel, resident.hip)
// spends a request on four crossings: workgroup 0 mirrors the request to the others,
// then layer 1 -> layer 2, layer 2 -> head, and one granule sweep per layer by a
// 16-output tile GEMV with an LDS reduction over 8 waves (profiles/r03_res_timeline.json:
// 1.0 us mirror, 1.7 us per layer, 1.2 us per hand-off). Here a request crosses
// workgroups twice, and each layer is a few hundred cycles:
//
//  * no mirror: every workgroup's polling wave (wave 0) polls the request ring in
//    device memory itself (the host writes it through the large-BAR mapping, so the
//    32 pollers read HBM, not PCIe; without large BAR the engine runs the r03 form);
//  * layer 0 in every workgroup ("local", as r03): compute lane c owns output c of
//    the 64 CW = H outputs, its F0 weight float4s in registers; one broadcast
//    ds_read_b128 of the observation row per float4;
//  * the sliced layers 1 .. NL - 2: workgroup p owns outputs [16 p, 16 p + 16); each
//    DPP row of 16 lanes (RPO = CW / 4 rows per output) holds the weights of its
//    output over 256 k, 16 consecutive k per lane, in registers for the kernel's life;
//    16 fma per lane, the row sum by DPP (a1_reduce), the two rows of an output joined
//    by one row_bcast:15 add;
//  * between sliced layers the outputs cross as 8-byte {tag, value} granules (the data
//    IS the flag: cdna_hip_programming.md Guideline 16 R2). Wave 0 of each workgroup
//    (the "communication wave", the poller) stores its workgroup's 16 outputs of a row
//    as one 128-byte line in ONE store instruction, sweeps all H granules of the row
//    (8 per lane) into LDS, and the compute waves read them after a barrier: one wave
//    per CU touches another workgroup's data (compute waves sweeping for themselves, 8
//    per CU, each output's granule stored by its own row's lane, lost granules of whole
//    waves under load: the line written piecewise by 8 waves);
//  * the head (<= 16 outputs) is split over the workgroups by k: workgroup p multiplies
//    its 16 last-layer outputs by the head's columns [16 p, 16 p + 16) (each row of the
//    last sliced layer: its output times the column, lane s for head output s, into
//    LDS) and its communication wave sums and publishes the 16 partials; workgroup 0 sums the P partials of each output in a fixed order
//    (the second and last crossing; its communication wave sweeps them), adds the bias,
//    applies the head's activation and the action epilogue, and answers as {epoch,
//    value} granules in host memory.
//
// Summation order (deterministic, within the 1e-5 contract of the fp64 oracle; not the
// MFMA path's order): layer 0 two packed fma chains per output; a sliced layer two
// packed chains per lane, the fixed DPP tree, then the row pair; the head per
// workgroup its 16 column products in column order, then the partials in workgroup
// order p = q + 4u (u ascending within each of four lane groups q, then q by xor 16,
// xor 32).
//
// Leaving: a LEAVE request header, idle_ticks without a request, a moved yield
// counter, or the launch's abort word (set by a communication wave whose granule sweep
// met a LEAVE tag or timed out) makes every polling wave leave; a leaving workgroup tags every
// granule slot it produces LEAVE, so a workgroup still waiting on one fails its sweep
// and leaves too. Every spin is bounded, so the grid always drains; workgroup 0 sets
// done = LEAVE after its own stores have drained (engine.cpp resident_serve).
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "resident_fn.hpp"

namespace go2pi {

namespace {

// a uniform value kept in an SGPR as it is (not reloaded from the program)
__device__ __forceinline__ int w_keep(int v) {
  v = __builtin_amdgcn_readfirstlane(v);
  asm volatile("" : "+s"(v));
  return v;
}
__device__ __forceinline__ float w_keep(float v) { return __int_as_float(w_keep(__float_as_int(v))); }

// rows 1 and 3 of each wave add lane 15 of rows 0 and 2 (every lane of a row holds
// the row's sum after a1_reduce): the two k halves of an output joined (RPO = 2)
__device__ __forceinline__ float w_pair_add(float v) {
  float r = v;
  asm volatile("s_nop 1\n\tv_add_f32_dpp %0, %1, %0 row_bcast:15 row_mask:0xa bank_mask:0xf" : "+v"(r) : "v"(v));
  return r;
}

// One wave's N granules per lane, g[i * S], i < N, re-read until every tag equals `tag`
// in every lane: 1 done, -1 a producer left (a LEAVE tag), 0 timeout (err set).
template <int N, int S>
__device__ __forceinline__ int w_sweep(const u64 *g, unsigned tag, float (&v)[N], unsigned *err, int lane) {
  u64 *gm = const_cast<u64 *>(g);
  for (unsigned spins = 0;; ++spins) {
    u64 x[N];
#pragma unroll
    for (int i = 0; i < N; ++i) x[i] = __hip_atomic_load(gm + i * S, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    bool ok = true, lv = false;
#pragma unroll
    for (int i = 0; i < N; ++i) {
      const unsigned t = (unsigned)(x[i] >> 32);
      ok &= t == tag;
      lv |= t == GO2PI_RES_LEAVE;
      v[i] = __uint_as_float((unsigned)x[i]);
    }
    if (__any(lv)) return -1;
    if (__all(ok)) return 1;
    if (spins > (1u << 22)) {
      if (lane == 0) __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      return 0;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}

// The polling wave's wait for the next request (every workgroup's own; the ring in
// device memory). D sweeps of the header and the first 63 request granules in flight,
// each checked when it lands; the yield counter and the launch's abort word ride along.
// 1: a request, its observation in x0 (prologue applied), e / B set; 0: leave.
template <int D, bool PRO>
__device__ __forceinline__ int w_poll(const u64 *q, int in_dim, unsigned last, u64 idle_ticks, unsigned *err,
                                      int lane, unsigned &e, int &B, const unsigned *yield, unsigned y0,
                                      const u64 *abortw, float *x0, int S, const Pro &pro, const ProK &pk,
                                      u64 (&v)[D], unsigned (&yv)[D], u64 (&av)[D]) {
  u64 *qm = const_cast<u64 *>(q);
  u64 *am = const_cast<u64 *>(abortw);
  const int npoll = min(1 + in_dim, 64);
  // the previous call's sweeps, landed long ago: used here, so their registers stay theirs
#pragma unroll
  for (int d = 0; d < D; ++d) asm volatile("" ::"v"(v[d]), "v"(yv[d]), "v"(av[d]));
  auto issue = [&](int d) {
    v[d] = __hip_atomic_load(qm + min(lane, npoll - 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    yv[d] = __hip_atomic_load(const_cast<unsigned *>(yield), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    av[d] = __hip_atomic_load(am, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  };
#pragma unroll
  for (int d = 0; d + 1 < D; ++d) issue(d);
  const u64 t0 = wall_clock64();
  for (;;) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
      issue((d + D - 1) % D);  // the newest sweep, before the oldest is looked at
      if (__builtin_amdgcn_readfirstlane(yv[d]) != y0) return 0;
      if (__builtin_amdgcn_readfirstlane((unsigned)av[d]) != 0u) return 0;
      const unsigned tag = __builtin_amdgcn_readfirstlane((unsigned)(v[d] >> 32));
      if (tag == GO2PI_RES_LEAVE) return 0;
      if (tag != 0u && tag != last) {
        const unsigned word = __builtin_amdgcn_readfirstlane((unsigned)v[d]);
        B = min(max((int)(word & 0xFFu), 1), GO2PI_SMALL_MAXB);
        const int n = B * in_dim;
        e = tag;
        if (1 + n <= npoll) {
          const bool ok = lane < 1 || lane > n || (unsigned)(v[d] >> 32) == tag;
          if (__all(ok)) {
            if (lane >= 1 && lane <= n) {
              const int b = (lane - 1) / in_dim, k = (lane - 1) - b * in_dim;
              const float x = __uint_as_float((unsigned)v[d]);
              x0[b * S + k] = PRO ? prologue(pro, pk, x) : x;
            }
            return 1;
          }
        } else {  // more granules than one sweep holds (B > 1)
          for (unsigned spins = 0;; ++spins) {
            bool ok = true, lv = false;
            for (int i = 1 + lane; i <= n; i += 64) {
              const u64 g = __hip_atomic_load(qm + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
              const unsigned t = (unsigned)(g >> 32);
              ok &= t == tag;
              lv |= t == GO2PI_RES_LEAVE;
              const int b = (i - 1) / in_dim, k = (i - 1) - b * in_dim;
              const float x = __uint_as_float((unsigned)g);
              x0[b * S + k] = PRO ? prologue(pro, x, k) : x;
            }
            if (__any(lv)) return 0;
            if (__all(ok)) return 1;
            if (spins > (1u << 22)) {
              if (lane == 0) __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
              return 0;
            }
          }
        }
      }
      if (wall_clock64() - t0 > idle_ticks) return 0;
    }
  }
}

// the float4 W[n][k .. k + 3] of dense layer L (packed fragment order, program.hpp);
// zero where k >= K_pad
__device__ __forceinline__ float4 w_ld(const DevLayer &L, int n, int k) {
  const float4 *W = reinterpret_cast<const float4 *>(L.w);
  float4 r = make_float4(0.f, 0.f, 0.f, 0.f);
  if (k < L.K_pad) r = W[((size_t)(k >> 4) * (L.N_pad >> 4) + (n >> 4)) * 64 + (n & 15) + 16 * ((k & 15) >> 2)];
  return r;
}

#ifdef GO2PI_DIAG_RESCLK
// (tools/res_timeline.py --form wide): wall-clock stamps of workgroups 0 and 17, 16 slots
// each per request: 0 request seen (communication wave), 1 layer 0 done (first compute
// wave), 2 + l sliced layer l's input in LDS (l >= 1: after the granule sweep), 6 the last
// sliced layer's outputs in LDS, 7 the head partials published, 8 every workgroup's
// partials gathered (workgroup 0), 9 the answer stored
#define W_STAMP(t, i)                                                                                  \
  do {                                                                                                 \
    if (P.stamps && tid == (t) && (wg == 0 || wg == 17))                                               \
      ((gu64_t *)P.stamps)[(size_t)(nreq & 511) * 32 + (wg ? 16 : 0) + (i)] = wall_clock64();          \
  } while (0)
#else
#define W_STAMP(t, i) \
  do {                \
  } while (0)
#endif

}  // namespace

// NL: dense layers (3 or 4: layer 0, NL - 2 sliced layers of H = 64 CW outputs, the head
// of <= 16 outputs). CW: compute waves (4 or 8; the grid is H / 16 workgroups). F0:
// layer 0's weight float4s per lane (K0_pad <= 4 F0). PRO: an observation prologue,
// applied by the communication wave as it stages the request.
// gran: [NL - 1][gstride] granules, zeroed before every launch: region r < NL - 3 the
// outputs of sliced layer r + 1 ([8][H]), region NL - 3 the head partials ([8][NP][16]),
// the last slot of region NL - 2 the launch's abort word.
//
// Wave 0 is the workgroup's communication wave: it polls the request ring, stores the
// workgroup's granules (each 128-byte line of 16 granules by one store instruction:
// written piecewise by several waves, 8 bytes each, some lines lost a wave's granules
// under load, and stale tags stayed in them), sweeps the granules of every workgroup
// into LDS, and in workgroup 0 gathers the head partials and answers. Only it reads or
// writes another workgroup's data (the one-polling-wave hand-off of
// cdna_hip_programming.md Guideline 16; the compute waves read LDS after a barrier).
template <int NL, int CW, int F0, bool PRO>
__global__ __launch_bounds__(64 * (1 + CW)) void policy_wide_kernel(const DevProgram *__restrict__ Pd,
                                                                    const u64 *req, u64 *actg, u64 *gran,
                                                                    int gstride, unsigned *err, unsigned *done,
                                                                    u64 idle_ticks, const unsigned *yield) {
  static_assert(NL >= 3 && NL <= 4 && (CW == 4 || CW == 8) && F0 >= 1 && F0 <= 16, "policy_wide_kernel shape");
  constexpr int H = 64 * CW;    // hidden width
  constexpr int NT = 64 * (1 + CW);
  constexpr int RPO = CW / 4;   // DPP rows per output of a sliced layer
  constexpr int NS = NL - 2;    // sliced layers
  constexpr int NP = H / 16;    // workgroups (partials per head output)
  constexpr int S0 = 4 * F0;    // layer 0's input row stride (floats)
  constexpr int MB = GO2PI_SMALL_MAXB;
  const DevProgram &P = *Pd;
  extern __shared__ float4 lds4[];
  float *x0 = reinterpret_cast<float *>(lds4);  // [8][S0] the observation rows (prologued, zero-padded)
  float *h0 = x0 + MB * S0;                     // [8][H] layer 0's outputs
  float *hh = h0 + MB * H;                      // [8][H] a sliced layer's outputs of every workgroup (swept)
  float *ho = hh + MB * H;                      // [8][16] this workgroup's outputs of a sliced layer
  float *pp = ho + MB * 16;                     // [8][16 columns][16 head outputs] its head products
  int *st = reinterpret_cast<int *>(pp + MB * 256);  // [0] leave [1] epoch [2] batch [3] fail
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wg = blockIdx.x;
  const int c = tid - 64;                 // compute lane (the communication wave: negative)
  const int s = c & 15, g = c >> 4;       // lane within its DPP row, the row
  const int o = g / RPO, kh = g % RPO;    // sliced layers: the row's output (of this workgroup's 16), k half
  const int kb = kh * 256 + 16 * s;       // ... and the lane's first k (16 consecutive)
  const int in_dim = P.in_dim, nout = P.out_dim;
  u64 *part = gran + (size_t)(NS - 1) * gstride;          // [8][NP][16] head partials
  u64 *abortw = gran + (size_t)(NL - 1) * gstride - 1;    // the launch's abort word
  unsigned nreq = 0;
  (void)nreq;

  // ---- weights in registers for the kernel's life (zero where k >= K_pad)
  const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
  float4 w0[F0], wm[NS][4];
  float b0 = 0.f, bm[NS], wh = 0.f, bh = 0.f;
  if (c >= 0) {
#pragma unroll
    for (int f = 0; f < F0; ++f) w0[f] = w_ld(P.L[0], c, 4 * f);
    b0 = P.L[0].bias[c];
#pragma unroll
    for (int l = 0; l < NS; ++l) {
#pragma unroll
      for (int f = 0; f < 4; ++f) wm[l][f] = w_ld(P.L[1 + l], 16 * wg + o, kb + 4 * f);
      bm[l] = P.L[1 + l].bias[16 * wg + o];
    }
    {  // the head's weight of output s at column 16 wg + o (the row's last-layer output)
      const float4 w = w_ld(P.L[NL - 1], s, (16 * wg + o) & ~3);
      const int r = o & 3;
      wh = r == 0 ? w.x : (r == 1 ? w.y : (r == 2 ? w.z : w.w));
    }
  } else {
#pragma unroll
    for (int f = 0; f < F0; ++f) w0[f] = z4;
#pragma unroll
    for (int l = 0; l < NS; ++l) {
#pragma unroll
      for (int f = 0; f < 4; ++f) wm[l][f] = z4;
      bm[l] = 0.f;
    }
    if (wg == 0 && lane < 16) bh = P.L[NL - 1].bias[lane];  // (the answer: workgroup 0's communication wave)
  }
  // the activations and the action epilogue, in SGPRs for the kernel's life
  int lact[NL];
  float lal[NL], lbe[NL];
#pragma unroll
  for (int l = 0; l < NL; ++l) {
    lact[l] = w_keep(P.L[l].act);
    lal[l] = w_keep(P.L[l].alpha);
    lbe[l] = w_keep(P.L[l].beta);
  }
  const int post_tanh = w_keep(P.post_tanh);
  const float clo = w_keep(P.clip_lo), chi = w_keep(P.clip_hi), pscale = w_keep(P.scale);
  // the communication wave: its lane's prologue constants (granule lane = column lane - 1)
  const Pro pro = PRO ? pro_of(P) : Pro{};
  const ProK pk = (PRO && wave == 0 && lane >= 1) ? pro_k(pro, (lane - 1) % in_dim) : ProK{0.f, 1.f, 1.f};
  for (int i = tid; i < MB * S0; i += NT) x0[i] = 0.f;
  if (tid == 0) st[3] = 0;
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): weights in registers before the first wait
  const unsigned y0 = __hip_atomic_load(const_cast<unsigned *>(yield), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();  // x0 cleared before the communication wave writes a row into it
  unsigned last = 0;
  constexpr int D = 2;
  u64 pv[D], pa[D];
  unsigned pyv[D];
#pragma unroll
  for (int d = 0; d < D; ++d) {
    pv[d] = pa[d] = 0ull;
    pyv[d] = 0u;
  }
  // a failed sweep (a producer left, or a timeout): the workgroup publishes nothing more
  // for this request, and every polling wave of the launch leaves
  auto fail = [&]() {
    if (lane == 0) {
      st[3] = 1;
      __hip_atomic_store(abortw, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  };
  // the communication wave stores rows b < B of src ([8][16] in LDS) as granules tagged t
  // at dst + b * rs + 16 wg (lane i: row i >> 4, output i & 15: each row's 16 granules,
  // one 128-byte line, from one store instruction)
  auto publish = [&](const float *src, u64 *dst, size_t rs, int B, unsigned t) {
#pragma unroll
    for (int i0 = 0; i0 < 16 * MB; i0 += 64) {
      const int i = i0 + lane, b = i >> 4;
      if (b < B)
        __hip_atomic_store(dst + (size_t)b * rs + 16 * wg + (i & 15), ((u64)t << 32) | __float_as_uint(src[i]),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  };
  for (;;) {
    if (wave == 0) {
      unsigned e = 0;
      int B = 1;
      const int got = (st[3] != 0) ? 0
                                   : w_poll<D, PRO>(req, in_dim, last, idle_ticks, err, lane, e, B, yield, y0,
                                                    abortw, x0, S0, pro, pk, pv, pyv, pa);
      W_STAMP(0, 0);
      if (lane == 0) {
        st[0] = !got;
        st[1] = (int)e;
        st[2] = B;
      }
    }
    lds_barrier();  // the request's rows are in x0
    const int3 sv = *reinterpret_cast<const int3 *>(st);
    if (sv.x) break;
    const unsigned e = (unsigned)sv.y;
    const int B = sv.z;
    last = e;
    // (every wave passes the same barriers per request; the communication wave has no
    // arithmetic, the compute waves no memory traffic beyond their own LDS)
    // ---- layer 0, all H outputs (lane c: output c)
    if (wave != 0) {
      const int A = lact[0];
      for (int b = 0; b < B; ++b) {
        f32x2 acc = {0.f, 0.f};
#pragma unroll
        for (int f = 0; f < F0; ++f) {
          const float4 x = *reinterpret_cast<const float4 *>(x0 + b * S0 + 4 * f);
          acc = __builtin_elementwise_fma(f32x2{x.x, x.y}, f32x2{w0[f].x, w0[f].y}, acc);
          acc = __builtin_elementwise_fma(f32x2{x.z, x.w}, f32x2{w0[f].z, w0[f].w}, acc);
        }
        h0[b * H + c] = act_fn(A, lal[0], lbe[0], acc.x + acc.y + b0);
      }
    }
    W_STAMP(64, 1);
    lds_barrier();  // layer 0's outputs visible
    // ---- the sliced layers
#pragma unroll
    for (int l = 0; l < NS; ++l) {  // layer 1 + l: its input in h0 (l = 0) or hh
      if (wave != 0 && st[3] == 0) {
        const int A = lact[1 + l];
        const float *X = l == 0 ? h0 : hh;
        for (int b = 0; b < B; ++b) {
          f32x2 acc = {0.f, 0.f};
#pragma unroll
          for (int f = 0; f < 4; ++f) {
            const float4 x = *reinterpret_cast<const float4 *>(X + b * H + kb + 4 * f);
            acc = __builtin_elementwise_fma(f32x2{x.x, x.y}, f32x2{wm[l][f].x, wm[l][f].y}, acc);
            acc = __builtin_elementwise_fma(f32x2{x.z, x.w}, f32x2{wm[l][f].z, wm[l][f].w}, acc);
          }
          float p[1] = {acc.x + acc.y};
          float v = a1_reduce<1>(p);
          if constexpr (RPO == 2) v = w_pair_add(v);
          if (l + 1 < NS) {
            if (s == 0 && kh == RPO - 1) ho[b * 16 + o] = act_fn(A, lal[1 + l], lbe[1 + l], v + bm[l]);
          } else if (kh == RPO - 1) {
            // the last sliced layer: its output o times the head's column, for every head
            // output s (lane s of the row; the row's lanes all hold the output)
            pp[(b * 16 + o) * 16 + s] = wh * act_fn(A, lal[1 + l], lbe[1 + l], v + bm[l]);
          }
        }
      }
      if (l + 1 < NS) {
        lds_barrier();  // this workgroup's outputs of layer 1 + l in ho
        if (wave == 0 && st[3] == 0) {
          // to every workgroup, then every workgroup's into hh (8 granules per lane per row)
          u64 *reg = gran + (size_t)l * gstride;
          publish(ho, reg, H, B, e + 1u + (unsigned)l);
          for (int b = 0; b < B; ++b) {
            float v8[H / 64];
            if (w_sweep<H / 64, 64>(reg + (size_t)b * H + lane, e + 1u + (unsigned)l, v8, err, lane) != 1) {
              fail();
              break;
            }
#pragma unroll
            for (int u = 0; u < H / 64; ++u) hh[b * H + lane + 64 * u] = v8[u];
          }
          if (l < 4) W_STAMP(0, 2 + l + 1);
        }
        lds_barrier();  // every workgroup's outputs of layer 1 + l in hh
      }
    }
    W_STAMP(64, 6);
    lds_barrier();  // the head products of this workgroup's 16 columns in pp
    if (wave == 0 && st[3] == 0) {
      // ---- the head's partial sums over this workgroup's 16 columns: lane 16 b' + j sums
      // output j's 16 products of row b (columns o = 0 .. 15 in order) and stores it; the
      // lanes of a row store its 16 partials, one 128-byte line, in one instruction
#pragma unroll
      for (int i0 = 0; i0 < 16 * MB; i0 += 64) {
        const int i = i0 + lane, b = i >> 4, j = i & 15;
        if (b < B) {
          const float *pr = pp + b * 256 + j;
          float a = 0.f;
#pragma unroll
          for (int oo = 0; oo < 16; ++oo) a += pr[oo * 16];
          __hip_atomic_store(part + ((size_t)b * NP + wg) * 16 + j, ((u64)(e + (unsigned)NL - 1u) << 32) | __float_as_uint(a),
                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
      W_STAMP(0, 7);
      // ---- workgroup 0: the partials of every workgroup summed, the answer
      if (wg == 0) {
        const int q = lane >> 4, j = lane & 15;
        for (int b = 0; b < B; ++b) {
          float pv2[NP / 4];
          if (w_sweep<NP / 4, 64>(part + ((size_t)b * NP + q) * 16 + j, e + (unsigned)NL - 1u, pv2, err, lane) != 1) {
            fail();
            break;
          }
          if (b == 0) W_STAMP(0, 8);
          float a = 0.f;
#pragma unroll
          for (int u = 0; u < NP / 4; ++u) a += pv2[u];
          a += __shfl_xor(a, 16);
          a += __shfl_xor(a, 32);
          if (lane < nout) {
            float y = act_fn(lact[NL - 1], lal[NL - 1], lbe[NL - 1], a + bh);
            if (post_tanh) y = tanhf(y);
            y = clip_nan(y, clo, chi) * pscale;
            int n = lane;
            asm volatile("" : "+v"(n));  // (the granule address formed here, not hoisted and spilled)
            __hip_atomic_store(actg + (size_t)b * nout + n, ((u64)e << 32) | __float_as_uint(y), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
          }
        }
        W_STAMP(0, 9);
      }
    }
    ++nreq;
  }
  // ---- leave: consumers still waiting on this workgroup's slots leave too (each line by
  // one store instruction)
  if (wave == 0) {
    const u64 lv = (u64)GO2PI_RES_LEAVE << 32;
#pragma unroll
    for (int i0 = 0; i0 < 16 * MB; i0 += 64) {
      const int i = i0 + lane, b = i >> 4, n = i & 15;
#pragma unroll
      for (int l = 0; l + 1 < NS; ++l)
        __hip_atomic_store(gran + (size_t)l * gstride + (size_t)b * H + 16 * wg + n, lv, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(part + ((size_t)b * NP + wg) * 16 + n, lv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (lane == 0) __hip_atomic_store(abortw, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  // every wave's stores (the answer granules among them) drained before the LEAVE done
  // word: a host that sees LEAVE and rescans finds a served request's answer
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (wg == 0 && tid == 0) __hip_atomic_store(done, GO2PI_RES_LEAVE, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// ---------------------------------------------------------------------------
// host side

// {NL, CW, F0} of program p when policy_wide_kernel serves it, else NL = 0: a dense
// policy of 3 or 4 layers whose hidden layers are all H = 256 or 512 wide, a head of
// <= 16 outputs and layer 0 of K_pad <= 64 (<= 48 for 4 layers of 512)
WideShape wide_shape(const DevProgram &p) {
  WideShape w{0, 0, 0};
  if (p.has_gru || p.nl < 3 || p.nl > 5 || p.L[p.nl - 1].N_pad != 16) return w;
  const int H = p.L[0].N_pad;
  if (H != 256 && H != 512) return w;
  for (int l = 1; l < p.nl; ++l)
    if (p.L[l].K_pad != H || (l + 1 < p.nl && p.L[l].N_pad != H)) return w;
  if (p.L[0].K_pad > 64 || p.in_dim > 63) return w;  // (one poll sweep holds the header and a row)
  if (p.nl == 5 || (p.nl == 4 && H == 512 && p.L[0].K_pad > 48)) return w;  // (their registers spilled)
  w.nl = p.nl;
  w.cw = H / 64;
  w.f0 = (w.nl == 4 && w.cw == 8) ? 12 : 16;  // (the instantiations launch_resident_wide runs)
  return w;
}

size_t wide_lds_bytes(const WideShape &w) {
  return sizeof(float) * ((size_t)GO2PI_SMALL_MAXB * (4 * w.f0 + 2 * 64 * w.cw + 16 + 256) + 4);
}

int launch_resident_wide(const DevProgram &p, const DevProgram *p_dev, const unsigned long long *req,
                         unsigned long long *actg, unsigned long long *gran, int gstride, unsigned *err, unsigned *done,
                         unsigned long long idle_ticks, const unsigned *yield, void *stream) {
  const WideShape w = wide_shape(p);
  if (!w.nl || !yield || gstride < GO2PI_SMALL_MAXB * 64 * w.cw) return (int)hipErrorInvalidValue;
  const size_t lds = wide_lds_bytes(w);
  const bool pro = p.pre_sub || p.pre_div || p.pre_mul || p.pre_clip;
  auto go = [&](auto kern) {
    hipLaunchKernelGGL(kern, dim3(4 * w.cw), dim3(64 * (1 + w.cw)), lds, reinterpret_cast<hipStream_t>(stream), p_dev,
                       req, actg, gran, gstride, err, done, idle_ticks, yield);
    return (int)hipGetLastError();
  };
  // the BASELINE policy's shape (48 -> 512^3 -> 12, no prologue) has its own
  // instantiation; every other shape the generic one (F0 = 16, the prologue applied)
  if (w.nl == 4 && w.cw == 8) return pro ? go(policy_wide_kernel<4, 8, 12, true>) : go(policy_wide_kernel<4, 8, 12, false>);
  if (w.cw == 8) return go(policy_wide_kernel<3, 8, 16, true>);
  if (w.nl == 3) return go(policy_wide_kernel<3, 4, 16, true>);
  return go(policy_wide_kernel<4, 4, 16, true>);
}

}  // namespace go2pi
