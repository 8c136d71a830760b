// Batched-path device code (templates) of the policy forward pass: shared by
// kernels.hip (generic bodies, small-batch kernels, dispatch) and the
// kernels_w4_t*.hip translation units (the 4-wave pipeline instantiations,
// compiled in parallel). See kernels.hip for the overview.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <type_traits>

#include "ctl_fn.hpp"
#include "device_fn.hpp"
#include "program.hpp"

namespace go2pi {

typedef float f32x4 __attribute__((ext_vector_type(4)));

// chunks ahead of the weight-fragment ring of the generic body at 4 waves per
// workgroup (2 and 3 measured slower: 40.2 / 42.2 vs 39.5 us)
#define GO2PI_RING_RD 1
// the 4-wave pipeline's ring depth by tiles per wave: a chunk is 4 * TPW MFMAs
// (32 cycles each), and a fragment must be issued >= ~1K cycles (an L2 round trip
// under load) before its MFMA
#ifndef GO2PI_W4_RD8
#define GO2PI_W4_RD8 1
#endif
#define GO2PI_W4_RD(TPW) ((TPW) >= 8 ? GO2PI_W4_RD8 : ((TPW) >= 4 ? 2 : 3))
#define GO2PI_FLAG_FLOATS 64  // LDS words for the per-wave layer hand-off flags (<= 64 waves)

// Diagnostic ablation builds only (tools/bound_probe.sh; outputs are wrong by design):
//   GO2PI_DIAG_NOMFMA  — replace each MFMA by one VALU fma (keeps the loads live)
//   GO2PI_DIAG_NOLOAD  — replace the weight loads by register arithmetic
__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
#ifdef GO2PI_DIAG_NOMFMA
  c.x = fmaf(a, b, c.x);
  return c;
#else
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
#endif
}

// ---------------------------------------------------------------------------
// Dense contraction over k-chunks [c0, c1) for TPW consecutive 16-col tiles.
// X: LDS activations [16][xs], W: this layer's fragments (chunk-major: the
// float4 stride between consecutive chunks of one tile is TL * 64).

// component j of a float4 (j a compile-time constant after unrolling)
__device__ __forceinline__ float f4c(const float4 &v, int j) {
  return j == 0 ? v.x : (j == 1 ? v.y : (j == 2 ? v.z : v.w));
}

// one weight fragment (GO2PI_DIAG_NOLOAD: register arithmetic instead, diagnostics)
__device__ __forceinline__ float4 load_frag(const float4 *p, int c, int cs, int i) {
#ifdef GO2PI_DIAG_NOLOAD
  const float v = __int_as_float(0x3c000000 ^ ((c * 7 + i) & 0xff));
  (void)p;
  (void)cs;
  return make_float4(v, v, v, v);
#else
  return p[c * cs];
#endif
}

// Weight-fragment stream over a buffer resource: one SGPR descriptor per layer,
// a per-lane byte offset per tile and the chunk offset folded into the scalar
// offset (sc1 or nt on these loads measured no change).
struct WStream {
  __amdgpu_buffer_rsrc_t r;
  __device__ __forceinline__ explicit WStream(const void *base)
      : r(__builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(base), (short)0, 0x7fffffff, 0x00020000)) {}
  __device__ __forceinline__ float4 ld(int voff, int soff) const {
#ifdef GO2PI_DIAG_NOLOAD
    const float v = __int_as_float(0x3c000000 ^ ((voff + soff) & 0xff));
    return make_float4(v, v, v, v);
#else
    return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0));
#endif
  }
};

// Schedule (measured on MI355X with tools/clock_probe.py, cycles per 16-robot
// workgroup of the 48->512^3->12 step): every tile's fragment for chunk c+1 is
// loaded right after that tile's 4 MFMAs of chunk c, so each wave keeps exactly
// one chunk in flight and its load issue is spread between MFMAs. Alternatives
// measured slower: no prefetch 110K (8 waves: 113K), one chunk ahead issued as a
// burst 123K/145K, three ahead 128K/144K, vs 104K-106K for this one; the
// MFMA-only ablation (no weight loads) is 97K-99K. sched_barrier(0) pins the
// order (hipcc otherwise sinks loads next to their uses). Tiles beyond T clamp
// to T - 1 (duplicate loads, results unused); loads past c1 clamp to c1 - 1.
// Requires (c1 - c0) % 4 == 0 (K padded to 64).
// (A flag hand-off between two wide layers instead of the workgroup barrier, and
// fragments prefetched across that barrier, both measured slower in this body:
// mlp512 47.8 vs 45.6 us, gru256 78.4 vs 76.4 us)
template <int TPW>
__device__ __forceinline__ void dense_acc(const float *X, int xs, const float4 *__restrict__ W, int TL, int t_first,
                                          int T, int c0, int c1, int lane, f32x4 (&acc)[TPW]) {
  const float *xrow = X + (lane & 15) * xs + ((lane >> 4) << 2);
  const WStream ws(W);
  int vo[TPW];                // per-lane byte offset of each tile's fragment in chunk 0
  const int csb = TL * 1024;  // bytes per chunk (all tiles)
#pragma unroll
  for (int i = 0; i < TPW; ++i) vo[i] = (min(t_first + i, T - 1) * 64 + lane) * 16;
  if (c0 >= c1) return;
  float4 cur[TPW];
#pragma unroll
  for (int i = 0; i < TPW; ++i) cur[i] = ws.ld(vo[i], c0 * csb);
  // the last 4-chunk group is peeled (TAIL) so no prefetch is issued past the end:
  // a trailing load would only be waited for by the epilogue
  // (A operands are read per 4-chunk group; double-buffering them across groups
  // measured slower: 100.4K vs 97.8K cycles per workgroup; fragments 2 chunks
  // ahead instead of 1 measured slower too: 98.1K vs 96.2K)
  auto group = [&](int c, auto tail_k) {
    constexpr bool TAIL = decltype(tail_k)::value;
    float4 a[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) a[u] = *reinterpret_cast<const float4 *>(xrow + (c + u) * 16);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int cn = c + u + 1;
      const bool LOAD = !(TAIL && u == 3);  // folded after unrolling
      float4 nxt[TPW];
      // k-step outer, tile inner: consecutive MFMAs hit different accumulators,
      // so one wave issues at the 32-cycle rate instead of waiting out the
      // 40-cycle dependent-accumulator latency. Each accumulator still sees its
      // k-steps in the same order, so results are bitwise unchanged. One
      // fragment load after every 4th MFMA: TPW loads spread over 4*TPW MFMAs.
#pragma unroll
      for (int j = 0; j < 4; ++j) {
#pragma unroll
        for (int i = 0; i < TPW; ++i) {
          acc[i] = mfma4(f4c(cur[i], j), f4c(a[u], j), acc[i]);
          const int s = j * TPW + i;
          if (LOAD && (s & 3) == 3) {
            __builtin_amdgcn_sched_barrier(0);
            nxt[s >> 2] = ws.ld(vo[s >> 2], cn * csb);
            __builtin_amdgcn_sched_barrier(0);
          }
        }
      }
      if (LOAD) {
#pragma unroll
        for (int i = 0; i < TPW; ++i) cur[i] = nxt[i];
      }
    }
  };
  int c = c0;
  for (; c + 4 < c1; c += 4) group(c, std::false_type{});
  group(c, std::true_type{});
}

// Contraction for one wave per SIMD (4 waves per workgroup): a wave owns TPW
// tiles over the full K and nothing on its SIMD competes for the matrix pipe,
// so the schedule must hide every latency by itself:
//   * weight fragments stream RD chunks ahead through a 4-slot register ring
//     (slot = chunk % 4): the fragment an MFMA consumes was issued >= RD - 1
//     chunks (>= (RD - 1) * 4 * TPW MFMAs) earlier;
//   * the A operand of chunk c + 1 is read from LDS during chunk c;
//   * loads are spread one per 4 MFMAs (sched_barrier pins them in place).
// The k-step / tile order is the same as dense_acc's, so every accumulator sees
// its k-steps in the same order: results are bitwise those of dense_acc.
// Requires C % 4 == 0 (K padded to 64) and C >= 4.
template <int TPW, int RD>
__device__ __forceinline__ void dense_acc_ring(const float *X, int xs, const float4 *__restrict__ W, int TL,
                                               int t_first, int T, int C, int lane, f32x4 (&acc)[TPW]) {
  static_assert(RD >= 1 && RD <= 3, "ring of 4 slots: at most 3 chunks ahead");
  const float *xrow = X + (lane & 15) * xs + ((lane >> 4) << 2);
  const WStream ws(W);
  int vo[TPW];                // per-lane byte offset of each tile's fragment in chunk 0
  const int csb = TL * 1024;  // bytes per chunk (all tiles)
#pragma unroll
  for (int i = 0; i < TPW; ++i) vo[i] = (min(t_first + i, T - 1) * 64 + lane) * 16;
  float4 f[4][TPW];
  float4 a[2];
#pragma unroll
  for (int d = 0; d < RD; ++d)
#pragma unroll
    for (int i = 0; i < TPW; ++i) f[d][i] = ws.ld(vo[i], d * csb);
  a[0] = *reinterpret_cast<const float4 *>(xrow);
  // one 4-chunk group; TAIL: the last one (no loads past C)
  auto group = [&](int c0, auto tail_k) {
    constexpr bool TAIL = decltype(tail_k)::value;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int c = c0 + u;
      if (!(TAIL && u == 3)) a[(u + 1) & 1] = *reinterpret_cast<const float4 *>(xrow + (c + 1) * 16);
      const bool LOAD = !(TAIL && u + RD >= 4);  // chunk c + RD exists (folded after unrolling)
      constexpr int NS = 4 * TPW;                 // MFMAs per chunk
#pragma unroll
      for (int j = 0; j < 4; ++j) {
#pragma unroll
        for (int i = 0; i < TPW; ++i) {
          acc[i] = mfma4(f4c(f[u][i], j), f4c(a[u & 1], j), acc[i]);
          const int s = j * TPW + i;
          if (LOAD && (s % (NS / TPW)) == (NS / TPW) - 1) {
            __builtin_amdgcn_sched_barrier(0);
            f[(u + RD) & 3][s / (NS / TPW)] = ws.ld(vo[s / (NS / TPW)], (c + RD) * csb);
            __builtin_amdgcn_sched_barrier(0);
          }
        }
      }
    }
  };
  int c0 = 0;
  for (; c0 + 4 < C; c0 += 4) group(c0, std::false_type{});
  group(c0, std::true_type{});
}

// Accumulator layout of the dense path ("output-major"): the weight fragment is
// the MFMA's A operand and the activations its B operand, so D = W_tile . X^T
// and lane l holds outputs n = 16t + 4(l >> 4) + r (r = 0..3) of robot l & 15:
// four consecutive outputs of one robot, i.e. one float4 of its activation row.
// (The product and the per-accumulator k order are those of X . W^T: results
// are bitwise the same as with the operands the other way round.)

// The bias is fetched before the contraction and added in the epilogue, so its
// load latency hides behind the MFMA loop instead of delaying the first MFMA.
template <int TPW>
__device__ __forceinline__ void load_bias(float4 (&bv)[TPW], const float *__restrict__ bias, int t_first, int T,
                                          int lane) {
#pragma unroll
  for (int i = 0; i < TPW; ++i)
    bv[i] = *reinterpret_cast<const float4 *>(bias + min(t_first + i, T - 1) * 16 + ((lane >> 4) << 2));
}

// Epilogue of a hidden layer: bias + activation, one float4 per tile and lane to
// the LDS activation row (one ds_write_b128 instead of four ds_write_b32); the
// activated values also go to `keep` (head fusion consumes them from registers).
// Epilogue of the final layer: bias + activation + post, valid rows/cols to HBM.
template <int TPW, bool KEEP = false>
__device__ __forceinline__ void dense_store(const DevProgram &P, const DevLayer &L, f32x4 (&acc)[TPW],
                                            const float4 (&bv)[TPW], int t_first, int T, int lane, bool last,
                                            float *Y, int ys, float *out, const CtlView ctl, int row0, int B,
                                            float4 (&keep)[TPW]) {
  const int rob = lane & 15, n0 = (lane >> 4) << 2;
  // fields read once (the final layer's stores would make every element reload them)
  const int LN = L.N;
  const Post po = post_of(P);
  with_act(L.act, [&](auto act_k) {
    constexpr int ACT = decltype(act_k)::value;
    const ActP ap{L.act, L.alpha, L.beta};
#pragma unroll
    for (int i = 0; i < TPW; ++i) {
      const int t = t_first + i;
      if (t >= T) continue;
      float4 v;
      v.x = act_t<ACT>(ap, acc[i][0] + bv[i].x);
      v.y = act_t<ACT>(ap, acc[i][1] + bv[i].y);
      v.z = act_t<ACT>(ap, acc[i][2] + bv[i].z);
      v.w = act_t<ACT>(ap, acc[i][3] + bv[i].w);
      if (!last) {
        *reinterpret_cast<float4 *>(Y + rob * ys + t * 16 + n0) = v;
        if constexpr (KEEP) keep[i] = v;
      } else {
        const int row = row0 + rob;
        if (row >= B) continue;
        if (ctl.on && LN == GO2PI_CTL_DOF) {  // controller tick: this lane's four joints at once
          const int n = t * 16 + n0;
          if (n < LN) {
            const float y[4] = {post_fn(po, v.x), post_fn(po, v.y), post_fn(po, v.z), post_fn(po, v.w)};
            ctl_store4(ctl, row, n, y);
          }
          continue;
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int n = t * 16 + n0 + r;
          if (n >= LN) continue;
          const float y = post_fn(po, f4c(v, r));
          if (ctl.on) ctl_store(ctl, row, n, y);  // controller tick: action post-processing
          else out[(size_t)row * LN + n] = y;
        }
      }
    }
  });
}

// HT > 0: "head fusion". The final, narrow layer HL (HT <= 2 output tiles, e.g.
// the 12 actions) is accumulated inside this layer: the wave's freshly stored
// tiles are exactly its K-chunks of HL, so it multiplies them (read back from
// LDS by the same wave) against HL's fragments, fetched before its MFMA loop.
// Partials are summed across waves in a fixed order by head_finish (below).
template <int TPW, int HT, int RD = 0>
__device__ __forceinline__ void dense_group(const DevProgram &P, const DevLayer &L, const float *X, float *Y, int xs,
                                            int t_first, int T, int C, int lane, bool last, float *out,
                                            const CtlView ctl, int row0, int B, const DevLayer *HL,
                                            f32x4 (&hacc)[HT > 0 ? HT : 1]) {
  constexpr int HN = HT > 0 ? HT : 1;
  f32x4 acc[TPW];
  float4 bv[TPW];
  float4 hw[HN][TPW];
  load_bias<TPW>(bv, L.bias, t_first, T, lane);
  if constexpr (HT > 0) {
    const float4 *HW = reinterpret_cast<const float4 *>(HL->w);
    const int HTL = HL->N_pad >> 4;  // head tiles (chunk-major fragments)
#pragma unroll
    for (int h = 0; h < HT; ++h)
#pragma unroll
      for (int i = 0; i < TPW; ++i) hw[h][i] = HW[((size_t)min(t_first + i, T - 1) * HTL + h) * 64 + lane];
  }
#pragma unroll
  for (int i = 0; i < TPW; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  // per-wave phase stamps inside layer 1: entry, contraction done, epilogue done
  [[maybe_unused]] const bool st = &L == &P.L[1] && lane == 0;
  [[maybe_unused]] const int sts = 16 + 3 * (threadIdx.x >> 6);
  GO2PI_STAMP(P, st, sts);
  if constexpr (RD > 0)
    dense_acc_ring<TPW, RD>(X, xs, reinterpret_cast<const float4 *>(L.w), L.N_pad >> 4, t_first, T, C, lane, acc);
  else
    dense_acc<TPW>(X, xs, reinterpret_cast<const float4 *>(L.w), L.N_pad >> 4, t_first, T, 0, C, lane, acc);
  GO2PI_STAMP(P, st, sts + 1);
  float4 yv[TPW];
  dense_store<TPW, (HT > 0)>(P, L, acc, bv, t_first, T, lane, last, Y, xs, out, ctl, row0, B, yv);
  GO2PI_STAMP(P, st, sts + 2);
  if constexpr (HT > 0) {
    // the head's B operand for k-chunk t_first + i is exactly the float4 this
    // lane just stored (its robot, k = 16t + 4(lane >> 4) + j): use the registers
#pragma unroll
    for (int i = 0; i < TPW; ++i) {
      if (t_first + i >= T) continue;
#pragma unroll
      for (int h = 0; h < HT; ++h) {
        hacc[h] = mfma4(hw[h][i].x, yv[i].x, hacc[h]);
        hacc[h] = mfma4(hw[h][i].y, yv[i].y, hacc[h]);
        hacc[h] = mfma4(hw[h][i].z, yv[i].z, hacc[h]);
        hacc[h] = mfma4(hw[h][i].w, yv[i].w, hacc[h]);
      }
    }
  }
}

template <int TPW>
__device__ __forceinline__ void dense_group(const DevProgram &P, const DevLayer &L, const float *X, float *Y, int xs,
                                            int t_first, int T, int C, int lane, bool last, float *out,
                                            const CtlView ctl, int row0, int B) {
  f32x4 none[1];
  dense_group<TPW, 0>(P, L, X, Y, xs, t_first, T, C, lane, last, out, ctl, row0, B, nullptr, none);
}

// Tiles of a wide layer split over the NW waves (full K per wave), optionally
// with the fused head (HT > 0). Barrier-free.
template <int NW, int HT>
__device__ __forceinline__ void dense_tiles(const DevProgram &P, const DevLayer &L, const float *X, float *Y, int xs,
                                            int wave, int lane, bool last, float *out, const CtlView ctl, int row0,
                                            int B, const DevLayer *HL, f32x4 (&hacc)[HT > 0 ? HT : 1]) {
  const int T = L.N_pad >> 4, C = L.K_pad >> 4;
  // largest tile group per pass: bounded so the accumulators fit the VGPR
  // budget of NW waves per CU (512 / (NW/4) registers per lane)
  // (2-tile groups at 8 waves measured slower: 50.5 vs 44.5 us)
  constexpr int G = NW >= 16 ? 2 : (NW >= 8 ? 4 : 8);
  // one wave per SIMD: the register-ring contraction (dense_acc_ring)
  constexpr int RD = NW == 4 ? GO2PI_RING_RD : 0;
  const int tpw = (T + NW - 1) / NW;
  int t = wave * tpw;
  const int t_end = min(t + tpw, T);
  for (; t + G <= t_end; t += G) {
    dense_group<G, HT, RD>(P, L, X, Y, xs, t, T, C, lane, last, out, ctl, row0, B, HL, hacc);
  }
  const int rem = t_end - t;
  if (G > 4 && rem > 4)
    dense_group<G, HT, RD>(P, L, X, Y, xs, t, t_end, C, lane, last, out, ctl, row0, B, HL, hacc);
  else if (G > 2 && rem > 2)
    dense_group<(G > 4 ? 4 : G), HT, RD>(P, L, X, Y, xs, t, t_end, C, lane, last, out, ctl, row0, B, HL, hacc);
  else if (rem == 2)
    dense_group<2, HT, RD>(P, L, X, Y, xs, t, t_end, C, lane, last, out, ctl, row0, B, HL, hacc);
  else if (rem == 1)
    dense_group<1, HT, RD>(P, L, X, Y, xs, t, t_end, C, lane, last, out, ctl, row0, B, HL, hacc);
}

// Layer with the final layer fused in (P.head_fuse = HT tiles): per-wave head
// partials go to LDS scratch; head_finish sums them after the layer barrier.
template <int NW, int HT>
__device__ __forceinline__ void dense_layer_head(const DevProgram &P, const DevLayer &L, const DevLayer &HL,
                                                 const float *X, float *Y, int xs, f32x4 *scratch, int wave,
                                                 int lane, int row0, int B) {
  f32x4 hacc[HT];
#pragma unroll
  for (int h = 0; h < HT; ++h) hacc[h] = f32x4{0.f, 0.f, 0.f, 0.f};
  dense_tiles<NW, HT>(P, L, X, Y, xs, wave, lane, false, nullptr, CtlView{}, row0, B, &HL, hacc);
#pragma unroll
  for (int h = 0; h < HT; ++h) scratch[(h * NW + wave) * 64 + lane] = hacc[h];
}

template <int NW>
__device__ __forceinline__ void head_finish(const DevProgram &P, const DevLayer &HL, const f32x4 *scratch, int wave,
                                            int lane, float *out, const CtlView ctl, int row0, int B) {
  const int T = HL.N_pad >> 4;
  if (wave >= T) return;
  f32x4 acc[1] = {scratch[(wave * NW) * 64 + lane]};
  for (int w = 1; w < NW; ++w) acc[0] += scratch[(wave * NW + w) * 64 + lane];  // fixed order: deterministic
  float4 bv[1];
  load_bias<1>(bv, HL.bias, wave, T, lane);
  float4 none[1];
  dense_store<1>(P, HL, acc, bv, wave, T, lane, true, nullptr, 0, out, ctl, row0, B, none);
}

// One dense layer for the whole workgroup (NW waves). Contains barriers only in
// the split-K branch, which every wave of the workgroup takes together.
template <int NW>
__device__ __forceinline__ void dense_layer(const DevProgram &P, const DevLayer &L, const float *X, float *Y, int xs,
                                            f32x4 *scratch, int wave, int lane, bool last, float *out,
                                            const CtlView ctl, int row0, int B) {
  const int T = L.N_pad >> 4, C = L.K_pad >> 4;
  if (T >= NW) {
    f32x4 none[1];
    dense_tiles<NW, 0>(P, L, X, Y, xs, wave, lane, last, out, ctl, row0, B, nullptr, none);
  } else {
    // narrow layer (e.g. the 12-action head): split K over waves, reduce in LDS
    const int ks = NW / T;
    const int t = wave % T, s = wave / T;
    f32x4 acc[1];
    float4 bv[1];
    load_bias<1>(bv, L.bias, t, T, lane);
    acc[0] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (s < ks) {
      const int C4 = C >> 2;  // split on 4-chunk boundaries (dense_acc unrolls by 4)
      const int c0 = 4 * ((s * C4) / ks), c1 = 4 * (((s + 1) * C4) / ks);
      dense_acc<1>(X, xs, reinterpret_cast<const float4 *>(L.w), T, t, T, c0, c1, lane, acc);
      if (s > 0) scratch[wave * 64 + lane] = acc[0];
    }
    __syncthreads();
    if (s == 0) {
      for (int s2 = 1; s2 < ks; ++s2) acc[0] += scratch[(t + s2 * T) * 64 + lane];
      float4 none[1];
      dense_store<1>(P, L, acc, bv, t, T, lane, last, Y, xs, out, ctl, row0, B, none);
    }
  }
}

// GRU cell (ONNX semantics, linear_before_reset = 1) for one 16-robot tile.
// X: LDS rows [16][xs] holding x in columns [0, I_pad); Hs: LDS hidden rows
// (stride xs). Writes h' to Y[:, 0:H]; the caller copies it back into Hs after
// a barrier (other waves still read Hs as their MFMA A operand here).
template <int GT>
__device__ __forceinline__ void gru_group(const DevGru &G, const float *X, const float *Hs, float *Y, int xs,
                                          int t_first, int lane) {
  const int Cx = G.I_pad >> 4, Ch = G.H >> 4, Cc = Cx + Ch;
  const float4 *W = reinterpret_cast<const float4 *>(G.w);
  const int col = lane & 15, r0 = (lane >> 4) << 2;
  f32x4 z[GT], r[GT], nx[GT], nh[GT];
  const WStream ws(W);
  int vo[GT];  // per-lane byte offset of tile t_first + i's z fragment in chunk 0 (r: +1 KiB, n: +2 KiB)
#pragma unroll
  for (int i = 0; i < GT; ++i) {
    const int j = (t_first + i) * 16 + col;
    const float bz = G.bzr[j], br = G.bzr[G.H + j], bx = G.bh[j], bh = G.bh[G.H + j];
    z[i] = f32x4{bz, bz, bz, bz};
    r[i] = f32x4{br, br, br, br};
    nx[i] = f32x4{bx, bx, bx, bx};
    nh[i] = f32x4{bh, bh, bh, bh};
    vo[i] = ((t_first + i) * 192 + lane) * 16;
  }
  const int csb = (G.H >> 4) * 192 * 16;  // bytes per chunk, chunk-major: [chunk][tile][gate][lane]
  const float *xrow = X + (lane & 15) * xs + ((lane >> 4) << 2);
  const float *hrow = Hs + (lane & 15) * xs + ((lane >> 4) << 2);
  // One stream over the concatenated [x | h] chunks, scheduled like dense_acc:
  // each gate fragment of chunk c+1 is loaded right after that gate's 4 MFMAs
  // of chunk c (x chunks feed z, r, n_x; h chunks feed z, r, n_h).
  float4 cz[GT], cr[GT], chh[GT];
#pragma unroll
  for (int i = 0; i < GT; ++i) {
    cz[i] = ws.ld(vo[i], 0);
    cr[i] = ws.ld(vo[i] + 1024, 0);
    chh[i] = ws.ld(vo[i] + 2048, 0);
  }
  auto step = [&](int c, const float4 &a, f32x4 (&third)[GT], int cn) {
    float4 nz[GT], nr[GT], nh3[GT];
    // k-step outer over the 3*GT independent gate accumulators (no back-to-back
    // dependent MFMA; per-accumulator k order unchanged), one gate-fragment load
    // after every 4th MFMA
#pragma unroll
    for (int j = 0; j < 4; ++j) {
#pragma unroll
      for (int i = 0; i < GT; ++i) {
        z[i] = mfma4(f4c(a, j), f4c(cz[i], j), z[i]);
        r[i] = mfma4(f4c(a, j), f4c(cr[i], j), r[i]);
        third[i] = mfma4(f4c(a, j), f4c(chh[i], j), third[i]);
#pragma unroll
        for (int g = 0; g < 3; ++g) {
          const int s = (j * GT + i) * 3 + g;
          if ((s & 3) == 3) {
            const int q = s >> 2, ti = q / 3, gi = q % 3;
            __builtin_amdgcn_sched_barrier(0);
            const float4 f = ws.ld(vo[ti] + 1024 * gi, cn * csb);
            if (gi == 0) nz[ti] = f;
            else if (gi == 1) nr[ti] = f;
            else nh3[ti] = f;
            __builtin_amdgcn_sched_barrier(0);
          }
        }
      }
    }
#pragma unroll
    for (int i = 0; i < GT; ++i) {
      cz[i] = nz[i];
      cr[i] = nr[i];
      chh[i] = nh3[i];
    }
    (void)c;
  };
  for (int c = 0; c < Cx; ++c) step(c, *reinterpret_cast<const float4 *>(xrow + c * 16), nx, c + 1);
  for (int c = 0; c < Ch; ++c)
    step(Cx + c, *reinterpret_cast<const float4 *>(hrow + c * 16), nh, min(Cx + c + 1, Cc - 1));
#pragma unroll
  for (int i = 0; i < GT; ++i) {
    const int j = (t_first + i) * 16 + col;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int row = r0 + e;
      const float zg = sigmoid_fast(z[i][e]);
      const float rg = sigmoid_fast(r[i][e]);
      const float hn = 2.f * sigmoid_fast(2.f * (nx[i][e] + rg * nh[i][e])) - 1.f;  // tanh, ~1e-7 abs
      const float ho = Hs[row * xs + j];
      Y[row * xs + j] = (1.f - zg) * hn + zg * ho;
    }
  }
}

// GRU cell with linear_before_reset = 0 (ONNX GRU-14: n = tanh(Wh x + Wbh + Rh (r . h)
// + Rbh); Keras reset_after=False) for one group of GT tiles. The reset gate must be
// complete for every hidden unit before the n contraction over h can start, so the
// cell runs in two passes over the [x | h] chunks with a workgroup barrier between:
//   pass 1 (PH = 1): r over [x | h]; r . h written to Y (every wave reads it in pass 2);
//   pass 2 (PH = 2): z over [x | h], n over [x | r . h]; h' = (1 - z) n + z h into hv.
// Three gate contractions in all, as with lbr = 1. The caller stores hv to Y after a
// second barrier (Y still holds r . h for the other waves until then).
template <int GT, int PH>
__device__ __forceinline__ void gru0_group(const DevGru &G, const float *X, const float *Hs, float *Y, int xs,
                                           int t_first, int lane, f32x4 (&hv)[GT]) {
  const int Cx = G.I_pad >> 4, Ch = G.H >> 4, H = G.H;
  const int col = lane & 15, r0 = (lane >> 4) << 2;
  const WStream ws(G.w);
  const int csb = Ch * 192 * 16;  // bytes per chunk: [chunk][tile][gate][lane]
  int vo[GT];
  f32x4 a0[GT], a1[GT];  // PH 1: r, -; PH 2: z, n
#pragma unroll
  for (int i = 0; i < GT; ++i) {
    const int j = (t_first + i) * 16 + col;
    vo[i] = ((t_first + i) * 192 + lane) * 16;
    if (PH == 1) {
      const float br = G.bzr[H + j];
      a0[i] = f32x4{br, br, br, br};
    } else {
      const float bz = G.bzr[j], bn = G.bh[j] + G.bh[H + j];
      a0[i] = f32x4{bz, bz, bz, bz};
      a1[i] = f32x4{bn, bn, bn, bn};
    }
  }
  const float *xrow = X + (lane & 15) * xs + ((lane >> 4) << 2);
  const float *hrow = Hs + (lane & 15) * xs + ((lane >> 4) << 2);
  const float *rrow = Y + (lane & 15) * xs + ((lane >> 4) << 2);
  for (int c = 0; c < Cx + Ch; ++c) {
    const bool xc = c < Cx;
    const float4 a = xc ? *reinterpret_cast<const float4 *>(xrow + c * 16)
                        : *reinterpret_cast<const float4 *>(hrow + (c - Cx) * 16);
    float4 an = a;
    if (PH == 2 && !xc) an = *reinterpret_cast<const float4 *>(rrow + (c - Cx) * 16);
    float4 f0[GT], f1[GT];
#pragma unroll
    for (int i = 0; i < GT; ++i) {
      f0[i] = ws.ld(vo[i] + (PH == 1 ? 1024 : 0), c * csb);  // r (PH 1) or z fragment
      if (PH == 2) f1[i] = ws.ld(vo[i] + 2048, c * csb);     // n fragment (W_h on x, R_h on h)
    }
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int i = 0; i < GT; ++i) {
        a0[i] = mfma4(f4c(a, j), f4c(f0[i], j), a0[i]);
        if (PH == 2) a1[i] = mfma4(f4c(an, j), f4c(f1[i], j), a1[i]);
      }
  }
#pragma unroll
  for (int i = 0; i < GT; ++i) {
    const int j = (t_first + i) * 16 + col;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int row = r0 + e;
      const float ho = Hs[row * xs + j];
      if (PH == 1) {
        Y[row * xs + j] = sigmoid_fast(a0[i][e]) * ho;
      } else {
        const float zg = sigmoid_fast(a0[i][e]);
        const float hn = 2.f * sigmoid_fast(2.f * a1[i][e]) - 1.f;  // tanh, ~1e-7 abs
        hv[i][e] = (1.f - zg) * hn + zg * ho;
      }
    }
  }
}

// lbr = 0 over the workgroup: one group of <= GM tiles per wave (the engine admits
// H <= 256 for lbr = 0, so tpw <= GM for every wave count); every wave passes both
// barriers.
template <int NW, int GM>
__device__ __forceinline__ void gru0_cell(const DevGru &G, const float *X, const float *Hs, float *Y, int xs,
                                          int wave, int lane) {
  const int Ht = G.H >> 4;
  const int tpw = (Ht + NW - 1) / NW;
  const int t = wave * tpw, n = max(0, min(tpw, Ht - t));
  f32x4 hv[GM];
  auto pass = [&](auto ph) {
    constexpr int PH = decltype(ph)::value;
    if (n == GM) gru0_group<GM, PH>(G, X, Hs, Y, xs, t, lane, hv);
    else if (GM >= 2 && n == 2) gru0_group<2, PH>(G, X, Hs, Y, xs, t, lane, reinterpret_cast<f32x4(&)[2]>(hv));
    else if (n >= 1) {
      for (int i = 0; i < n; ++i)
        gru0_group<1, PH>(G, X, Hs, Y, xs, t + i, lane, reinterpret_cast<f32x4(&)[1]>(hv[i]));
    }
  };
  pass(std::integral_constant<int, 1>{});
  __syncthreads();  // r . h complete in Y
  pass(std::integral_constant<int, 2>{});
  __syncthreads();  // every wave done reading r . h
  const int col = lane & 15, r0 = (lane >> 4) << 2;
  for (int i = 0; i < n; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) Y[(r0 + e) * xs + (t + i) * 16 + col] = hv[i][e];
}

template <int NW>
__device__ __forceinline__ void gru_cell(const DevGru &G, const float *X, const float *Hs, float *Y, int xs,
                                         int wave, int lane) {
  if (G.lbr == 0) {
    constexpr int GM0 = NW >= 16 ? 1 : (NW >= 8 ? 2 : 4);
    gru0_cell<NW, GM0>(G, X, Hs, Y, xs, wave, lane);
    return;
  }
  const int Ht = G.H >> 4;
  const int tpw = (Ht + NW - 1) / NW;
  int t = wave * tpw;
  const int t_end = min(t + tpw, Ht);
  constexpr int GM = NW >= 16 ? 1 : (NW >= 8 ? 2 : 4);  // VGPR budget per wave count
  for (; t + GM <= t_end; t += GM) gru_group<GM>(G, X, Hs, Y, xs, t, lane);
  if (GM > 2)
    for (; t + 2 <= t_end; t += 2) gru_group<2>(G, X, Hs, Y, xs, t, lane);
  for (; t < t_end; ++t) gru_group<1>(G, X, Hs, Y, xs, t, lane);
}

// LSTM cell (ONNX semantics: gates i, o, f, c; f = sigmoid, g = h = tanh; no
// peepholes) for one 16-robot tile, generic body (any wave count). X: LDS rows
// holding x in [0, I_pad); Hs: LDS hidden rows (stride xs). h' goes to Y[:, 0:H]
// (the caller copies it into Hs after a barrier, as for the GRU); the cell state c
// is elementwise per (robot, unit), so the lane that owns a unit reads c from and
// writes c' to the engine's state rows in HBM (hidden[row][H + j]) itself.
template <int GT>
__device__ __forceinline__ void lstm_group(const DevGru &G, const float *X, const float *Hs, float *Y, int xs,
                                           int t_first, int lane, float *hidden, int row0, int B) {
  const int Cx = G.I_pad >> 4, Ch = G.H >> 4, Cc = Cx + Ch, H = G.H;
  const int col = lane & 15, r0 = (lane >> 4) << 2;
  f32x4 acc[4][GT];  // gates i, o, f, c
  const WStream ws(G.w);
  int vo[GT];  // per-lane byte offset of tile t_first + i's gate-i fragment in chunk 0 (gate g: + g KiB)
#pragma unroll
  for (int i = 0; i < GT; ++i) {
    const int j = (t_first + i) * 16 + col;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const float b = G.bzr[g * H + j];
      acc[g][i] = f32x4{b, b, b, b};
    }
    vo[i] = ((t_first + i) * 4 * 64 + lane) * 16;
  }
  const int csb = Ch * 4 * 1024;  // bytes per chunk: [chunk][tile][gate][lane]
  const float *xrow = X + (lane & 15) * xs + ((lane >> 4) << 2);
  const float *hrow = Hs + (lane & 15) * xs + ((lane >> 4) << 2);
  float4 cur[4][GT];
#pragma unroll
  for (int i = 0; i < GT; ++i)
#pragma unroll
    for (int g = 0; g < 4; ++g) cur[g][i] = ws.ld(vo[i] + 1024 * g, 0);
  for (int c = 0; c < Cc; ++c) {
    const float4 a = c < Cx ? *reinterpret_cast<const float4 *>(xrow + c * 16)
                            : *reinterpret_cast<const float4 *>(hrow + (c - Cx) * 16);
    float4 nxt[4][GT];
    const int cn = min(c + 1, Cc - 1);
#pragma unroll
    for (int i = 0; i < GT; ++i)
#pragma unroll
      for (int g = 0; g < 4; ++g) nxt[g][i] = ws.ld(vo[i] + 1024 * g, cn * csb);
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int i = 0; i < GT; ++i)
#pragma unroll
        for (int g = 0; g < 4; ++g) acc[g][i] = mfma4(f4c(a, j), f4c(cur[g][i], j), acc[g][i]);
#pragma unroll
    for (int i = 0; i < GT; ++i)
#pragma unroll
      for (int g = 0; g < 4; ++g) cur[g][i] = nxt[g][i];
  }
  const int sw = G.sw;
#pragma unroll
  for (int i = 0; i < GT; ++i) {
    const int j = (t_first + i) * 16 + col;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int row = r0 + e, grow = row0 + row;
      const float ig = sigmoid_fast(acc[0][i][e]), og = sigmoid_fast(acc[1][i][e]);
      const float fg = sigmoid_fast(acc[2][i][e]);
      const float cg = 2.f * sigmoid_fast(2.f * acc[3][i][e]) - 1.f;  // tanh, ~1e-7 abs
      const float c_old = grow < B ? hidden[(size_t)grow * sw + H + j] : 0.f;
      const float c_new = fg * c_old + ig * cg;
      Y[row * xs + j] = og * (2.f * sigmoid_fast(2.f * c_new) - 1.f);
      if (grow < B) hidden[(size_t)grow * sw + H + j] = c_new;
    }
  }
}

template <int NW>
__device__ __forceinline__ void lstm_cell(const DevGru &G, const float *X, const float *Hs, float *Y, int xs,
                                          int wave, int lane, float *hidden, int row0, int B) {
  const int Ht = G.H >> 4;
  const int tpw = (Ht + NW - 1) / NW;
  int t = wave * tpw;
  const int t_end = min(t + tpw, Ht);
  constexpr int GM = NW >= 8 ? 1 : 2;  // VGPR budget per wave count (four gates)
  for (; t + GM <= t_end; t += GM) lstm_group<GM>(G, X, Hs, Y, xs, t, lane, hidden, row0, B);
  for (; t < t_end; ++t) lstm_group<1>(G, X, Hs, Y, xs, t, lane, hidden, row0, B);
}

// ---------------------------------------------------------------------------
// Uniform-MLP pipeline at one wave per SIMD (4 waves per workgroup; the engine
// selects it for policies whose hidden layers are all 64 * TPW wide, TPW = 2, 4
// or 8, with the final layer fused as the head). Wave w owns output tiles
// [t0, t0 + TPW) of EVERY hidden layer, t0 = w * TPW, over the full K.
//
//  * Weight stream: a 4-slot register ring of MFMA A-operand fragments (slot =
//    consumption index k & 3) filled RD chunks ahead by buffer loads, one per 4
//    MFMAs. It runs across layer boundaries: the tail of layer l issues layer
//    l + 1's first RD chunks, layer 0's go out before the observation barrier.
//  * Register hand-off: the k-chunks of layer l + 1 that a wave produced itself
//    (chunks t0 .. t0 + TPW - 1: its own output tiles of layer l) are consumed
//    FIRST and straight from registers: the epilogue value of tile t0 + i (one
//    float4 per lane = the MFMA B operand for that chunk) feeds chunk i, and the
//    epilogue of tile i + 1 is interleaved with chunk i's MFMAs (sched_group
//    pattern). Each tile also goes to LDS for the other waves. The remaining
//    chunks are read from LDS in rotated order (t0 + k mod C) after ONE wait on
//    the other waves' per-layer flags (LDS words) — no workgroup barrier between
//    layers, and the epilogue runs beside the MFMA pipe instead of in front of it.
//  * WAR safety of the two LDS activation buffers: a wave writes layer l + 1's
//    tiles into the buffer layer l read only after it has seen every wave's
//    layer-l flag, which each wave sets after it finished reading that buffer
//    (its layer l contraction).
// Numerics: every accumulator is an fp32 fma chain over its K in a fixed
// per-output order (own chunks first, then rotated): identical for every robot
// row, so sharded and unsharded runs stay bitwise equal; the order differs from
// the generic body's, which the tolerance-based parity tests cover.

// one chunk (16 k) of MFMAs for the wave's TPW tiles: A = ring slot S, B = b
// (4 k-steps in its components); LOAD: after every 4th MFMA the next fragment of
// the chunk RD ahead goes into slot (S + RD) & 3 at byte offset soff of ws. PIN:
// sched_barrier around each load (the LDS phase); otherwise the caller's
// sched_group pattern places it (the own phase).
// Load spacing: one fragment load after every LSP-th MFMA, so the chunk's TPW
// loads are issued over its first LSP * TPW MFMAs (the earlier they go out, the
// longer the last tile's fragment has before its MFMA in the next chunk).
#ifndef GO2PI_W4_LSP
#define GO2PI_W4_LSP 2
#endif
template <int TPW, int S, int RD, bool LOAD, bool PIN>
__device__ __forceinline__ void w4_chunk(f32x4 (&acc)[TPW], float4 (&f)[4][TPW], const float4 &b, const WStream &ws,
                                         const int (&vo)[TPW], int soff) {
  constexpr int LSP = GO2PI_W4_LSP;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
#pragma unroll
    for (int i = 0; i < TPW; ++i) {
      acc[i] = mfma4(f4c(f[S][i], j), f4c(b, j), acc[i]);
      const int s = j * TPW + i;
      if (LOAD && s % LSP == LSP - 1 && s / LSP < TPW) {
        if constexpr (PIN) __builtin_amdgcn_sched_barrier(0);
        f[(S + RD) & 3][s / LSP] = ws.ld(vo[s / LSP], soff);
        if constexpr (PIN) __builtin_amdgcn_sched_barrier(0);
      }
    }
  }
}

// bias + activation of one 16 x 16 tile (output-major: one float4 per lane)
template <int ACT>
__device__ __forceinline__ float4 w4_epi(const ActP &ap, const f32x4 &acc, const float4 &bv) {
  float4 v;
  v.x = act_t<ACT>(ap, acc[0] + bv.x);
  v.y = act_t<ACT>(ap, acc[1] + bv.y);
  v.z = act_t<ACT>(ap, acc[2] + bv.z);
  v.w = act_t<ACT>(ap, acc[3] + bv.w);
  return v;
}

// The lean kernel's Elu epilogue (ACTC == 1: Elu with alpha = 1, the exported
// policies'): the bias is already in the accumulator (BIN: the first MFMA of each
// tile took it as its C operand), and the x * log2(e) and e - 1 steps run as
// packed pairs. Per element the value of act_t<1> with alpha = 1 (x > 0 ? x :
// exp2(x * log2 e) - 1), the same bits for the same x (x = -0 aside, below).
// (A select-free form, max(x, clamp(e, 0, 1) - 1), measured 0.4 % faster but maps
// a NaN to -1 where ONNX Elu propagates it: rejected, DESIGN §4.1. The integer min
// below propagates it.)
// r06 A/B (profiles/r06_ab_epi.txt): VGPR accumulators + the integer min, mlp512
// 35.43 -> 35.02-35.12 us, GRU-256 tick 57.0 -> 56.4-56.5 us.
typedef float f32x2 __attribute__((ext_vector_type(2)));
template <bool BIN>
__device__ __forceinline__ float4 w4_epi_elu1(const f32x4 &acc, const float4 &bv) {
  f32x2 x01 = {acc[0], acc[1]}, x23 = {acc[2], acc[3]};
  if constexpr (!BIN) {
    x01 += f32x2{bv.x, bv.y};
    x23 += f32x2{bv.z, bv.w};
  }
  // (r06: the accumulators are VGPRs, the pipeline units are built with
  // -amdgpu-mfma-vgpr-form: no accvgpr read in front of each element, and no copy)
  const f32x2 L = {1.4426950408889634f, 1.4426950408889634f};
  const f32x2 t01 = x01 * L, t23 = x23 * L;
  f32x2 e01 = {__builtin_amdgcn_exp2f(t01.x), __builtin_amdgcn_exp2f(t01.y)};
  f32x2 e23 = {__builtin_amdgcn_exp2f(t23.x), __builtin_amdgcn_exp2f(t23.y)};
  e01 -= 1.f;
  e23 -= 1.f;
  // The select x > 0 ? x : e - 1 as one signed-integer min of the bit patterns (r06,
  // one v_min_i32 instead of a compare and a select): x > 0 (and +inf, and a NaN of
  // either sign) has e - 1 >= x with the same sign, so the smaller pattern is x; x <= 0
  // has x <= e - 1 <= 0, and negative patterns order by magnitude, so the min is e - 1
  // (x = -inf: -1). Bitwise the compare + select's result except at x = -0, which
  // gives -0 where the select gives +0.
  auto imin = [](float a, float b) {
    return __int_as_float(__builtin_elementwise_min(__float_as_int(a), __float_as_int(b)));
  };
  float4 v;
  v.x = imin(x01.x, e01.x);
  v.y = imin(x01.y, e01.y);
  v.z = imin(x23.x, e23.x);
  v.w = imin(x23.y, e23.y);
  return v;
}

// Chunks k in [k0, C) of a layer from the LDS activation rows X, chunk
// c = (kb + k) mod C, ring slots from K0S on (slot of chunk k0 + u = (K0S + u) & 3).
// Groups of 4 chunks, the last one NT chunks long ((C - k0) % 4 == NT % 4). NEXT:
// past the layer's own chunks the ring loads NL's chunks (kbn + d) mod Cn, d < RD
// (NL's consumption order), into the slots that follow: NL starts at slot
// (K0S + C - k0) & 3, which must be the slot NL's own phase starts on.
template <int TPW, int RD, int K0S, int NT, bool NEXT>
__device__ __forceinline__ void w4_lds_phase(const float *X, int xs, int lane, int C, int kb, int k0,
                                             const WStream &ws, int csb, const WStream &wn, int csn, int kbn, int Cn,
                                             const int (&vo)[TPW], f32x4 (&acc)[TPW], float4 (&f)[4][TPW]) {
  static_assert(K0S >= 0 && K0S <= 3 && NT >= 1 && NT <= 4 && RD <= NT, "phase shape");
  const float *xrow = X + (lane & 15) * xs + ((lane >> 4) << 2);
  auto chunk_of = [&](int k) {
    const int c = kb + k;
    return c >= C ? c - C : c;
  };
  auto next_of = [&](int d) {
    const int c = kbn + d;
    return c >= Cn ? c - Cn : c;
  };
  float4 a[2];
  a[0] = *reinterpret_cast<const float4 *>(xrow + chunk_of(k0) * 16);
  // one group of 4 chunks from k = g (slots K0S .. K0S + 3, mod 4); TAIL: the last
  auto group = [&](int g, auto tail_k) {
    constexpr bool TAIL = decltype(tail_k)::value;
    auto step = [&](auto u_k) {
      constexpr int U = decltype(u_k)::value;
      constexpr int S = (K0S + U) & 3;
      constexpr int N = TAIL ? NT : 4;  // chunks in this group
      if constexpr (U < N) {
        const int k = g + U;
        if (U + 1 < N || !TAIL) a[(U + 1) & 1] = *reinterpret_cast<const float4 *>(xrow + chunk_of(k + 1) * 16);
        constexpr bool OWN = !(TAIL && U + RD >= N);  // chunk k + RD is this layer's
        if constexpr (OWN)
          w4_chunk<TPW, S, RD, true, true>(acc, f, a[U & 1], ws, vo, chunk_of(k + RD) * csb);
        else if constexpr (NEXT)
          w4_chunk<TPW, S, RD, true, true>(acc, f, a[U & 1], wn, vo, next_of(U + RD - N) * csn);
        else
          w4_chunk<TPW, S, RD, false, true>(acc, f, a[U & 1], ws, vo, 0);
      }
    };
    step(std::integral_constant<int, 0>{});
    step(std::integral_constant<int, 1>{});
    step(std::integral_constant<int, 2>{});
    step(std::integral_constant<int, 3>{});
  };
  int g = k0;
  for (; g + NT < C; g += 4) group(g, std::false_type{});
  group(g, std::true_type{});
}

// Bounded wait until every OTHER wave has published epoch ep (an LDS word per
// wave). A protocol failure must not hang the GPU: past the bound the kernel
// reports through P.err (the engine raises it at the next sync) and goes on.
template <int NW = 4>
__device__ __forceinline__ void w4_wait(const int *flags, int wave, int ep, int lane, unsigned *err) {
  for (int it = 0;; ++it) {
    const int f = lane < NW && lane != wave ? __hip_atomic_load(flags + lane, __ATOMIC_RELAXED,
                                                                __HIP_MEMORY_SCOPE_WORKGROUP)
                                           : ep;
    if (__ballot(f < ep) == 0ull) break;
    if (it == (1 << 22)) {  // ~ seconds
      if (lane == 0 && err) __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      break;
    }
    __builtin_amdgcn_s_sleep(1);
  }
  asm volatile("" ::: "memory");  // the LDS reads of the other waves' tiles stay after the wait
}

// GRU cell as the pipeline's front stage (one wave per SIMD): wave w owns hidden
// tiles [w * GT, (w + 1) * GT) (H = 64 * GT) over the concatenated [x | h] chunks
// (Cx = I_pad / 16 and Ch = H / 16, both multiples of 4: the engine pads I to 64).
// The same register ring and buffer-load stream as the dense layers (RD = 1,
// loads every 2 MFMAs), B operand one chunk ahead from LDS, output-major
// accumulators (the gate fragment is the A operand): lane l holds units
// 16t + 4(l >> 4) + e of robot l & 15, so the old h and the new h' move as one
// float4 per tile. Gate math as gru_group (ONNX GRU, linear_before_reset = 1).
// h' goes to Y rows and to hn (registers) for the caller. The caller has issued
// the direct-to-LDS loads of x and h; this stage issues its first chunk's
// fragments, waits for everything OLDER than them (the LDS-DMA), then barriers,
// so the fragment latency overlaps the staging. Gate biases are added after the
// contraction (accumulators start at zero), so their loads wait nowhere.
// mid(): called between the contraction and the epilogue (the caller issues the next
// stage's first loads there, so their latency overlaps the gate math).
template <int GT, class Mid>
__device__ __forceinline__ void w4_gru(const DevGru &G, const float *X, const float *Hs, float *Y, int xs, int wave,
                                       int lane, float4 (&hn)[GT], unsigned long long *st, Mid &&mid) {
  GO2PI_STAMP_AT(st, wave == 0 && lane == 0, 43);  // GRU stage marks (wave 0): 43 entry, 44 contraction, 45 epilogue
  constexpr int NF = 3 * GT;  // gate fragments per chunk
  constexpr int NM = 4 * NF;  // MFMAs per chunk
  const int Cx = G.I_pad >> 4, Ch = G.H >> 4;
  const int t0 = wave * GT, u0 = (lane >> 4) << 2;
  const WStream ws(G.w);
  const int csb = Ch * 3 * 1024;  // bytes per chunk (all tiles, three gates)
  int vo[GT];                     // per-lane byte offset of tile t0 + i's z fragment in chunk 0 (r +1 KiB, n +2 KiB)
#pragma unroll
  for (int i = 0; i < GT; ++i) vo[i] = ((t0 + i) * 3 * 64 + lane) * 16;
  // x chunks that hold data: Cxe = ceil(I / 16) (the packing pads x to whole 4-chunk
  // groups; a 48-wide observation leaves chunk 3 all zeros, skipped here: its 4 * NF
  // MFMAs are 1/20 of GRU-256's stage). With Cxe = 3 mod 4 the ring starts on slot 1
  // so that the h chunks start on slot 0 and keep their 4-chunk groups.
  const int Cxe = (G.I + 15) >> 4;
  f32x4 z[GT], r[GT], nx[GT], nh[GT];
  float4 bz[GT], br[GT], bx[GT], bh[GT];
  const float *xrow = X + (lane & 15) * xs + u0;
  const float *hrow = Hs + (lane & 15) * xs + u0;
  auto run = [&](auto k0_k) {
    constexpr int K0S = decltype(k0_k)::value;  // ring slot of chunk 0
    float4 f[4][NF];
    asm volatile("" ::: "memory");  // the caller's LDS-DMA stays ahead of the NF loads
#pragma unroll
    for (int q = 0; q < NF; ++q) f[K0S][q] = ws.ld(vo[q / 3] + (q % 3) * 1024, 0);
    wg_barrier_vm<NF>();  // the x / h rows (LDS-DMA) have landed; chunk 0's fragments stay in flight
#pragma unroll
    for (int i = 0; i < GT; ++i) {
      const int j = (t0 + i) * 16 + u0;
      bz[i] = *reinterpret_cast<const float4 *>(G.bzr + j);
      br[i] = *reinterpret_cast<const float4 *>(G.bzr + G.H + j);
      bx[i] = *reinterpret_cast<const float4 *>(G.bh + j);
      bh[i] = *reinterpret_cast<const float4 *>(G.bh + G.H + j);
      z[i] = r[i] = nx[i] = nh[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    float4 a[2];
    a[K0S & 1] = *reinterpret_cast<const float4 *>(xrow);
    // chunk c (slot S); XPH: an x chunk (the third gate accumulates n_x, else n_h);
    // NEXT: a chunk follows, cn (its B operand and fragments are fetched here); NX:
    // that chunk is an x chunk (else an h chunk). One fixed source row per
    // instantiation keeps the B-operand read a single ds_read_b128.
    auto chunk = [&](auto s_k, auto xph_k, auto next_k, auto nx_k, int c, int cn) {
      constexpr int S = decltype(s_k)::value;
      constexpr bool XPH = decltype(xph_k)::value, NEXT = decltype(next_k)::value, NX = decltype(nx_k)::value;
      if constexpr (NEXT) {
        if constexpr (NX) a[(S + 1) & 1] = *reinterpret_cast<const float4 *>(xrow + cn * 16);
        else a[(S + 1) & 1] = *reinterpret_cast<const float4 *>(hrow + (cn - Cx) * 16);
      }
      const float4 b = a[S & 1];
#pragma unroll
      for (int m = 0; m < NM; ++m) {
        const int jk = m / NF, i = (m % NF) / 3, g = m % 3;
        const float wv = f4c(f[S][i * 3 + g], jk), bk = f4c(b, jk);
        if (g == 0) z[i] = mfma4(wv, bk, z[i]);
        else if (g == 1) r[i] = mfma4(wv, bk, r[i]);
        else if (XPH) nx[i] = mfma4(wv, bk, nx[i]);
        else nh[i] = mfma4(wv, bk, nh[i]);
        if (NEXT && (m & 1) == 1 && (m >> 1) < NF) {
          const int q = m >> 1;
          __builtin_amdgcn_sched_barrier(0);
          f[(S + 1) & 3][q] = ws.ld(vo[q / 3] + (q % 3) * 1024, cn * csb);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
    };
    using T_ = std::true_type;
    using F_ = std::false_type;
    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;
    using I2 = std::integral_constant<int, 2>;
    using I3 = std::integral_constant<int, 3>;
    int c = 0;
    if constexpr (K0S == 1) {  // a leading group of 3 x chunks (slots 1-3)
      if (Cxe > 3) {
        chunk(I1{}, T_{}, T_{}, T_{}, 0, 1);
        chunk(I2{}, T_{}, T_{}, T_{}, 1, 2);
        chunk(I3{}, T_{}, T_{}, T_{}, 2, 3);
        c = 3;
      } else {
        chunk(I1{}, T_{}, T_{}, T_{}, 0, 1);
        chunk(I2{}, T_{}, T_{}, T_{}, 1, 2);
        chunk(I3{}, T_{}, T_{}, F_{}, 2, Cx);  // the next chunk is the first h chunk
        c = Cxe;
      }
    }
    if (c < Cxe) {
      for (; c + 4 < Cxe; c += 4) {
        chunk(I0{}, T_{}, T_{}, T_{}, c, c + 1);
        chunk(I1{}, T_{}, T_{}, T_{}, c + 1, c + 2);
        chunk(I2{}, T_{}, T_{}, T_{}, c + 2, c + 3);
        chunk(I3{}, T_{}, T_{}, T_{}, c + 3, c + 4);
      }
      chunk(I0{}, T_{}, T_{}, T_{}, c, c + 1);
      chunk(I1{}, T_{}, T_{}, T_{}, c + 1, c + 2);
      chunk(I2{}, T_{}, T_{}, T_{}, c + 2, c + 3);
      chunk(I3{}, T_{}, T_{}, F_{}, c + 3, Cx);  // the next chunk is the first h chunk
    }
    for (c = Cx; c + 4 < Cx + Ch; c += 4) {
      chunk(I0{}, F_{}, T_{}, F_{}, c, c + 1);
      chunk(I1{}, F_{}, T_{}, F_{}, c + 1, c + 2);
      chunk(I2{}, F_{}, T_{}, F_{}, c + 2, c + 3);
      chunk(I3{}, F_{}, T_{}, F_{}, c + 3, c + 4);
    }
    chunk(I0{}, F_{}, T_{}, F_{}, c, c + 1);
    chunk(I1{}, F_{}, T_{}, F_{}, c + 1, c + 2);
    chunk(I2{}, F_{}, T_{}, F_{}, c + 2, c + 3);
    chunk(I3{}, F_{}, F_{}, F_{}, c + 3, c + 3);
  };
  if ((Cxe & 3) == 3) run(std::integral_constant<int, 1>{});
  else run(std::integral_constant<int, 0>{});
  GO2PI_STAMP_AT(st, wave == 0 && lane == 0, 44);
  mid();
  float *yrow = Y + (lane & 15) * xs + t0 * 16 + u0;
#pragma unroll
  for (int i = 0; i < GT; ++i) {
    const float4 ho = *reinterpret_cast<const float4 *>(hrow + (t0 + i) * 16);
    float o[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float zg = sigmoid_fast(z[i][e] + f4c(bz[i], e));
      const float rg = sigmoid_fast(r[i][e] + f4c(br[i], e));
      const float nxe = nx[i][e] + f4c(bx[i], e), nhe = nh[i][e] + f4c(bh[i], e);
      const float hv = 2.f * sigmoid_fast(2.f * (nxe + rg * nhe)) - 1.f;  // tanh, ~1e-7 abs
      o[e] = (1.f - zg) * hv + zg * f4c(ho, e);
    }
    hn[i] = make_float4(o[0], o[1], o[2], o[3]);
    *reinterpret_cast<float4 *>(yrow + i * 16) = hn[i];
  }
  GO2PI_STAMP_AT(st, wave == 0 && lane == 0, 45);
}

// LSTM cell as the pipeline's front stage (one wave per SIMD), the sibling of
// w4_gru: wave w owns hidden tiles [w * GT, (w + 1) * GT) (H = 64 * GT) over the
// concatenated [x | h] chunks, four gate fragments per (chunk, tile) streamed by
// the same register ring (RD = 1, a load every 2 MFMAs), output-major
// accumulators: lane l holds units 16t + 4(l >> 4) + e of robot l & 15. The cell
// state c of exactly those units lives in the caller's registers (c, in / out):
// it is elementwise, so no other wave ever needs it and across the ticks of a
// sequence it never leaves the CU. h' goes to Y rows and to hn.
template <int GT, class Mid>
__device__ __forceinline__ void w4_lstm(const DevGru &G, const float *X, const float *Hs, float *Y, int xs, int wave,
                                        int lane, float4 (&hn)[GT], float4 (&c)[GT], Mid &&mid) {
  constexpr int NF = 4 * GT;  // gate fragments per chunk
  constexpr int NM = 4 * NF;  // MFMAs per chunk
  const int Cx = G.I_pad >> 4, Ch = G.H >> 4, H = G.H;
  const int t0 = wave * GT, u0 = (lane >> 4) << 2;
  const WStream ws(G.w);
  const int csb = Ch * 4 * 1024;  // bytes per chunk (all tiles, four gates)
  int vo[GT];
#pragma unroll
  for (int i = 0; i < GT; ++i) vo[i] = ((t0 + i) * 4 * 64 + lane) * 16;
  // x chunks that hold data (as w4_gru: the all-zero padding chunk is skipped)
  const int Cxe = (G.I + 15) >> 4;
  f32x4 acc[4][GT];
  const float *xrow = X + (lane & 15) * xs + u0;
  const float *hrow = Hs + (lane & 15) * xs + u0;
  auto run = [&](auto k0_k) {
    constexpr int K0S = decltype(k0_k)::value;  // ring slot of chunk 0
    float4 f[4][NF];
    asm volatile("" ::: "memory");  // the caller's LDS-DMA stays ahead of the NF loads
#pragma unroll
    for (int q = 0; q < NF; ++q) f[K0S][q] = ws.ld(vo[q / 4] + (q % 4) * 1024, 0);
    wg_barrier_vm<NF>();  // the x / h rows (LDS-DMA) have landed; chunk 0's fragments stay in flight
#pragma unroll
    for (int i = 0; i < GT; ++i)
#pragma unroll
      for (int g = 0; g < 4; ++g) acc[g][i] = f32x4{0.f, 0.f, 0.f, 0.f};
    float4 a[2];
    a[K0S & 1] = *reinterpret_cast<const float4 *>(xrow);
    // chunk cc (slot S); NEXT: a chunk follows, cn; NX: cn is an x chunk
    auto chunk = [&](auto s_k, auto next_k, auto nx_k, int cc, int cn) {
      constexpr int S = decltype(s_k)::value;
      constexpr bool NEXT = decltype(next_k)::value, NX = decltype(nx_k)::value;
      if constexpr (NEXT) {
        if constexpr (NX) a[(S + 1) & 1] = *reinterpret_cast<const float4 *>(xrow + cn * 16);
        else a[(S + 1) & 1] = *reinterpret_cast<const float4 *>(hrow + (cn - Cx) * 16);
      }
      const float4 b = a[S & 1];
#pragma unroll
      for (int m = 0; m < NM; ++m) {
        const int jk = m / NF, i = (m % NF) / 4, g = m % 4;
        acc[g][i] = mfma4(f4c(f[S][i * 4 + g], jk), f4c(b, jk), acc[g][i]);
        if (NEXT && (m & 1) == 1 && (m >> 1) < NF) {
          const int q = m >> 1;
          __builtin_amdgcn_sched_barrier(0);
          f[(S + 1) & 3][q] = ws.ld(vo[q / 4] + (q % 4) * 1024, cn * csb);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
      (void)cc;
    };
    using T_ = std::true_type;
    using F_ = std::false_type;
    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;
    using I2 = std::integral_constant<int, 2>;
    using I3 = std::integral_constant<int, 3>;
    int cc = 0;
    if constexpr (K0S == 1) {  // a leading group of 3 x chunks (slots 1-3)
      if (Cxe > 3) {
        chunk(I1{}, T_{}, T_{}, 0, 1);
        chunk(I2{}, T_{}, T_{}, 1, 2);
        chunk(I3{}, T_{}, T_{}, 2, 3);
        cc = 3;
      } else {
        chunk(I1{}, T_{}, T_{}, 0, 1);
        chunk(I2{}, T_{}, T_{}, 1, 2);
        chunk(I3{}, T_{}, F_{}, 2, Cx);  // the next chunk is the first h chunk
        cc = Cxe;
      }
    }
    if (cc < Cxe) {
      for (; cc + 4 < Cxe; cc += 4) {
        chunk(I0{}, T_{}, T_{}, cc, cc + 1);
        chunk(I1{}, T_{}, T_{}, cc + 1, cc + 2);
        chunk(I2{}, T_{}, T_{}, cc + 2, cc + 3);
        chunk(I3{}, T_{}, T_{}, cc + 3, cc + 4);
      }
      chunk(I0{}, T_{}, T_{}, cc, cc + 1);
      chunk(I1{}, T_{}, T_{}, cc + 1, cc + 2);
      chunk(I2{}, T_{}, T_{}, cc + 2, cc + 3);
      chunk(I3{}, T_{}, F_{}, cc + 3, Cx);  // the next chunk is the first h chunk
    }
    for (cc = Cx; cc + 4 < Cx + Ch; cc += 4) {
      chunk(I0{}, T_{}, F_{}, cc, cc + 1);
      chunk(I1{}, T_{}, F_{}, cc + 1, cc + 2);
      chunk(I2{}, T_{}, F_{}, cc + 2, cc + 3);
      chunk(I3{}, T_{}, F_{}, cc + 3, cc + 4);
    }
    chunk(I0{}, T_{}, F_{}, cc, cc + 1);
    chunk(I1{}, T_{}, F_{}, cc + 1, cc + 2);
    chunk(I2{}, T_{}, F_{}, cc + 2, cc + 3);
    chunk(I3{}, F_{}, F_{}, cc + 3, cc + 3);
  };
  if ((Cxe & 3) == 3) run(std::integral_constant<int, 1>{});
  else run(std::integral_constant<int, 0>{});
  mid();
  float *yrow = Y + (lane & 15) * xs + t0 * 16 + u0;
#pragma unroll
  for (int i = 0; i < GT; ++i) {
    const int j = (t0 + i) * 16 + u0;
    const float4 bi = *reinterpret_cast<const float4 *>(G.bzr + j);
    const float4 bo = *reinterpret_cast<const float4 *>(G.bzr + H + j);
    const float4 bf = *reinterpret_cast<const float4 *>(G.bzr + 2 * H + j);
    const float4 bc = *reinterpret_cast<const float4 *>(G.bzr + 3 * H + j);
    float o[4], cn[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float ig = sigmoid_fast(acc[0][i][e] + f4c(bi, e));
      const float og = sigmoid_fast(acc[1][i][e] + f4c(bo, e));
      const float fg = sigmoid_fast(acc[2][i][e] + f4c(bf, e));
      const float cg = 2.f * sigmoid_fast(2.f * (acc[3][i][e] + f4c(bc, e))) - 1.f;  // tanh, ~1e-7 abs
      cn[e] = fg * f4c(c[i], e) + ig * cg;
      o[e] = og * (2.f * sigmoid_fast(2.f * cn[e]) - 1.f);
    }
    c[i] = make_float4(cn[0], cn[1], cn[2], cn[3]);
    hn[i] = make_float4(o[0], o[1], o[2], o[3]);
    *reinterpret_cast<float4 *>(yrow + i * 16) = hn[i];
  }
}

// Launch-critical values of the pipeline, read in ONE scalar burst from the
// program's hot block (program.hpp) at kernel start. Layer l's fragments are
// found from the arena base: every dense layer is packed back to back (engine.cpp),
// layer 0 is c0 k-chunks of 4 * TPW tiles, each hidden layer 4 * TPW chunks of
// 4 * TPW tiles, so no per-layer descriptor is read during the step (a scalar
// load outstanding at an LDS-read wait costs its whole latency: both count on
// lgkmcnt).
struct W4Hot {
  const float *l0w, *hw, *hb, *bpack;
  unsigned *err;
  int nbias, head_n, c0, hid_act, head_act;
  float hid_alpha, head_alpha;
  int post_plain;
  float hid_beta, head_beta;
  int in_dim = 0;  // the lean controller tick (PL && CTL): the observation width, from a preloaded argument
};

__device__ __forceinline__ W4Hot w4_hot(const DevProgram &P) {
  return W4Hot{P.l0_w,     P.head_w,  P.head_bias, P.bpack,    P.err_hot,   P.nbias,
               P.head_n,   P.c0,      P.hid_act,   P.head_act, P.hid_alpha, P.head_alpha, P.post_plain,
               P.hid_beta, P.head_beta};
}

// f(integral_constant<activation>): A >= 0 a compile-time activation (the lean
// kernel's instantiation for the policy's one hidden activation: no dispatch, one
// straight-line body the scheduler can interleave), A < 0 the runtime kind `act`.
template <int A, class F>
__device__ __forceinline__ void act_dispatch(int act, F &&f) {
  if constexpr (A >= 0) {
    (void)act;
    f(std::integral_constant<int, A>{});
  } else {
    with_act(act, f);
  }
}

// fragments of hidden layer l (l >= 1) of a TPW pipeline (arena layout above)
template <int TPW, int NW = 4>
__device__ __forceinline__ const float *w4_layer_w(const W4Hot &h, int l) {
  constexpr int CH = NW * TPW;
  return h.l0w + (size_t)(h.c0 + (l - 1) * CH) * CH * 256;
}

// Layer 0's first RD chunks of the wave's TPW tiles into the register ring (slots
// K0S ..): the loads w4_step starts a step with.
template <int TPW, int C0M, int NW = 4>
__device__ __forceinline__ void w4_prefill(const float *l0w, float4 (&f)[4][TPW], int wave, int lane) {
  constexpr int RD = GO2PI_W4_RD(TPW), CSB = NW * TPW * 1024, K0S = (4 - C0M) & 3;
  const WStream w0(l0w);
#pragma unroll
  for (int d = 0; d < RD; ++d)
#pragma unroll
    for (int i = 0; i < TPW; ++i) f[(K0S + d) & 3][i] = w0.ld(((wave * TPW + i) * 64 + lane) * 16, d * CSB);
}

// One policy step of the pipeline (the observation tile is being staged into bufA).
// pre: the ring already filled by w4_prefill and the biases' direct-to-LDS copy
// already issued (a recurrent policy does both behind its cell's contraction).
// X0: layer 0's input rows (the observation tile, or a GRU's h'); Y0: the other
// activation buffer (layer 0's outputs). PL: no action epilogue (post_fn is the
// identity: the lean kernel). C0M: layer 0's k-chunk count mod 4 (0, or 3 for
// a 48- or 98-wide observation padded to 16 rather than 64): layer 0 starts on
// ring slot (4 - C0M) & 3 so that its last chunk uses slot 3 and layer 1 starts on
// slot 0 as always.
template <int TPW, int HT, bool CTL, bool PL, int C0M, int ACTC = -1, int NHC = 0, int NW = 4>
__device__ __forceinline__ void w4_step(const DevProgram &P, const W4Hot &hot0, float *X0, float *Y0, int S,
                                        f32x4 *scratch, int *flags, float *lbias, int &ep, int wave, int lane,
                                        float *ac, const CtlView cv, int row0, int B, const DevCtl &ctl,
                                        const CtlLds &CL, int step, const float4 (&ring)[4][TPW], bool pre) {
  W4Hot hot = hot0;
  constexpr int RD = GO2PI_W4_RD(TPW);
  constexpr int CH = NW * TPW;    // k-chunks of every layer after the first (= output tiles of a hidden layer)
  constexpr int CSB = CH * 1024;  // bytes per k-chunk of a hidden layer's (and layer 0's) fragments
  constexpr int K0S = (4 - C0M) & 3, NT0 = C0M ? C0M : 4;  // layer 0: first ring slot, chunks in its last group
  static_assert(C0M == 0 || C0M == 3, "layer 0 chunk count mod 4");
  // register hand-off between layers for 4 and 8 tiles per wave; at 2 tiles per
  // wave (a 128-wide policy such as the shipped model) a layer's own phase is too
  // short to cover the other waves' epilogues, and an epilogue + barrier + natural
  // chunk order measured faster (9.9 vs 11.0 us per 4096-robot step)
  constexpr bool HO = TPW >= 4;
  // compile-time Elu (alpha 1): each hidden layer's bias enters as the C operand of
  // the tile's first MFMA (the fp32 chain starts at b instead of adding it after
  // the sum), and the epilogue is w4_epi_elu1
  constexpr bool BIN = ACTC == 1;
  const int t0 = wave * TPW;
  const int kb1 = HO ? t0 : 0;  // first k-chunk of every layer after the first
  // hidden layers (the fused head follows them); NHC > 0: a compile-time count, the
  // layer loop fully unrolled (a runtime loop carries the ring registers through
  // phi copies at its head, which wait for every fragment load in flight)
  const int nh = NHC > 0 ? NHC : hot.nbias / (16 * CH);
  int vo[TPW];              // per-lane byte offset of each own tile's fragment in chunk 0 (every layer)
#pragma unroll
  for (int i = 0; i < TPW; ++i) vo[i] = ((t0 + i) * 64 + lane) * 16;
  // every hidden layer's bias into LDS once, by direct-to-LDS loads in flight with
  // the observation tile's (read per tile by ds_read: off the vmcnt chain of the
  // weight stream, whose waits would otherwise cover them); the head's bias to registers
  if (step == 0 && !pre) glds_copy(lbias, hot.bpack, hot.nbias, wave, lane, NW);
  float4 hbv[1];  // the head's bias: fetched with the head's fragments (load_head)
  float4 f[4][TPW];
  asm volatile("" ::: "memory");  // the DMA and bias loads stay ahead of the ring's first loads
  if (pre) {
#pragma unroll
    for (int d = 0; d < RD; ++d)
#pragma unroll
      for (int i = 0; i < TPW; ++i) f[(K0S + d) & 3][i] = ring[(K0S + d) & 3][i];
  } else {
    w4_prefill<TPW, C0M, NW>(hot.l0w, f, wave, lane);
  }
  if constexpr (PL) {
    // the lean kernel: the program's remaining fields are loaded only now, behind the
    // observation, bias and first fragment loads (their round trip overlaps those)
    asm volatile("" ::: "memory");
    hot.hw = P.head_w;
    hot.hb = P.head_bias;
    hot.err = P.err_hot;
    hot.head_n = P.head_n;
    hot.hid_act = P.hid_act;
    hot.head_act = P.head_act;
    hot.hid_alpha = P.hid_alpha;
    hot.head_alpha = P.head_alpha;
    hot.hid_beta = P.hid_beta;
    hot.head_beta = P.head_beta;
  }
  GO2PI_STAMP(P, threadIdx.x == 0 && step == 0, 42);
  bool ctl_here = false;
  if constexpr (CTL) {
    // controller tick without a recurrent cell (fused_body ctl_late): the tick's raw rows
    // (direct-to-LDS, issued at kernel start) and the biases land behind the ring's
    // loads, which stay in flight; then the observation is assembled into X0 and
    // published to the caller's rows, and an LDS-only barrier hands X0 over
    ctl_here = step == 0 && (PL || !P.has_gru);  // (the lean kernel has no recurrent cell)
    if (ctl_here) {
      // (the lean tick: no program field, ctl_q_plain; otherwise its loads land behind the wait)
      const CtlQ cq = PL ? ctl_q_plain(ctl, hot.in_dim, 16 * hot.c0) : ctl_q(P, ctl);
      // r05: two waits. The direct-to-LDS loads went out as q0 | state, joystick and
      // action rows | previous observation rows (ctl_lds_load) | the hidden biases, then
      // the ring's fragments: the first wait lets this wave's observation, bias and ring
      // loads stay in flight, so the blocks that need only the state / joystick / action
      // rows are assembled while the observation rows land; the
      // second (inside the assembly) waits for those before vel_cmd and the shift pass.
      const int nrows = min(GO2PI_TILE_ROWS, B - row0);
      const int ind = PL ? hot.in_dim : P.in_dim;  // (the lean tick: no program round trip in front of the wait)
      const int later = glds_count(nrows * ind, wave, NW) + (step == 0 && !pre ? glds_count(hot.nbias, wave, NW) : 0);
      vm_wait_rt(later + RD * TPW);
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      GO2PI_STAMP(P, threadIdx.x == 0, 5);
      ctl_assemble_split<true>(P, CL, cq, ctl.joy != nullptr, nrows, X0, S, ctl.obs + (size_t)row0 * P.in_dim,
                               threadIdx.x, NW * 64, [] { wg_barrier_vm<RD * TPW>(); });
      lds_barrier();
    }
  }
  // layer 0's input rows are complete in X0 and the biases in LDS (this wave's
  // direct-to-LDS loads, older than the ring's); the ring's loads stay in flight
  // (NW = 8: vmcnt(0). The count RD * TPW assumes the ring's loads were issued after
  // the staging loads, but loads through a __restrict__ const pointer are invariant and
  // the compiler may sink them below this barrier: with run-time branches after it (an
  // r05 issue-priority experiment) it did, vmcnt(RD * TPW) waited for nothing, and rows
  // staged by waves 4-7 were read before they landed.)
  if (!ctl_here) wg_barrier_vm<NW == 8 ? 0 : RD * TPW>();
  GO2PI_STAMP(P, threadIdx.x == 0 && step == 0, 4);
  if constexpr (CTL) {
    if (ctl.status && (int)threadIdx.x < min(GO2PI_TILE_ROWS, B - row0)) ctl.status[row0 + threadIdx.x] = CL.nanf[threadIdx.x];
    GO2PI_STAMP(P, threadIdx.x == 0, 15);
  }
  // the head's fragments (final layer, fused): fetched before the last hidden layer's LDS phase
  float4 hw[HT][TPW];
  auto load_head = [&] {
    load_bias<1>(hbv, hot.hb, wave < HT ? wave : 0, HT, lane);
    const float4 *HW = reinterpret_cast<const float4 *>(hot.hw);
#pragma unroll
    for (int h = 0; h < HT; ++h)
#pragma unroll
      for (int i = 0; i < TPW; ++i) hw[h][i] = HW[((size_t)(t0 + i) * HT + h) * 64 + lane];
  };
  if (nh == 1) load_head();
  // layer 0: the observation tile, natural chunk order; the tail fetches layer 1's own chunks
  f32x4 acc[TPW];
  const float *brow = lbias + t0 * 16 + ((lane >> 4) << 2);  // this lane's bias float4 of tile t0, layer 0
  float4 bv[TPW];
#pragma unroll
  for (int i = 0; i < TPW; ++i) bv[i] = *reinterpret_cast<const float4 *>(brow + i * 16);
#pragma unroll
  for (int i = 0; i < TPW; ++i) acc[i] = BIN ? f32x4{bv[i].x, bv[i].y, bv[i].z, bv[i].w} : f32x4{0.f, 0.f, 0.f, 0.f};
  {
    const WStream ws(hot.l0w);
    if (nh > 1) {
      const WStream wn(w4_layer_w<TPW, NW>(hot, 1));
      w4_lds_phase<TPW, RD, K0S, NT0, true>(X0, S, lane, hot.c0, 0, 0, ws, CSB, wn, CSB, kb1, CH, vo, acc, f);
    } else {
      w4_lds_phase<TPW, RD, K0S, NT0, false>(X0, S, lane, hot.c0, 0, 0, ws, CSB, ws, 0, 0, 1, vo, acc, f);
    }
  }
  // pipeline stamps: 6 + l = wave 0 done with hidden layer l, 6 + nh = head barrier;
  // 16 + 3w + min(l, 2) = wave w done with hidden layer l
  GO2PI_STAMP(P, lane == 0 && step == 0, 16 + 3 * wave);
  GO2PI_STAMP(P, lane == 0 && step == 0 && wave == 0, 6);
  float *Y = Y0;  // where the previous layer's activations go
  const ActP ap{hot.hid_act, hot.hid_alpha, hot.hid_beta};
  constexpr int kHidUnroll = NHC > 0 ? NHC : 1;
#pragma unroll kHidUnroll
  for (int l = 1; l < nh; ++l) {
    const bool more = l + 1 < nh;
    const WStream ws(w4_layer_w<TPW, NW>(hot, l)), wn(w4_layer_w<TPW, NW>(hot, more ? l + 1 : l));
    float4 bvn[TPW];
#pragma unroll
    for (int i = 0; i < TPW; ++i) bvn[i] = *reinterpret_cast<const float4 *>(brow + l * CH * 16 + i * 16);
    f32x4 accn[TPW];
#pragma unroll
    for (int i = 0; i < TPW; ++i)
      accn[i] = BIN ? f32x4{bvn[i].x, bvn[i].y, bvn[i].z, bvn[i].w} : f32x4{0.f, 0.f, 0.f, 0.f};
    float *yrow = Y + (lane & 15) * S + t0 * 16 + ((lane >> 4) << 2);
    // publish this wave's layer l-1 tiles (after its own LDS stores) for the other waves
    auto publish = [&] {
      ++ep;
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's tile stores are in LDS
      if (lane == 0) __hip_atomic_store(flags + wave, ep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    };
    // layer 1 sub-phases per wave: 28 + 3w + {own phase done, wait done, LDS phase done}
    [[maybe_unused]] const bool sub = lane == 0 && step == 0 && l == 1;
    {
    // own phase: layer l-1's epilogue for all the wave's tiles (to registers and LDS),
    // publish, then layer l's MFMAs over those chunks with the B operand from registers
    // (!HO: the epilogue to LDS, then a workgroup barrier)
    act_dispatch<ACTC>(hot.hid_act, [&](auto act_k) {
      constexpr int ACT = decltype(act_k)::value;
      float4 v[TPW];
#pragma unroll
      for (int i = 0; i < TPW; ++i) {
        if constexpr (ACTC == 1) v[i] = w4_epi_elu1<BIN>(acc[i], bv[i]);
        else v[i] = w4_epi<ACT>(ap, acc[i], bv[i]);
      }
#pragma unroll
      for (int i = 0; i < TPW; ++i) *reinterpret_cast<float4 *>(yrow + i * 16) = v[i];
      GO2PI_STAMP(P, sub, 46 + wave);  // layer 1's epilogue issued (before the publish)
      constexpr bool LATEPUB = HO && PL;
      if constexpr (LATEPUB) {
        // the lean kernel publishes after its first own chunk: the publish's
        // lgkmcnt(0) then finds the tile stores landed instead of holding the MFMAs
        // behind them (mlp512 35.55 -> 35.43 us median, profiles/r03_ab_latepub.json;
        // in the GRU body it measured 60.09 -> 60.63 us per tick and no change over
        // 100-tick sequences, profiles/r03_ab_latepub_gru.json: it keeps the early flag)
        [&]<int... I>(std::integer_sequence<int, I...>) {
          ((w4_chunk<TPW, (I & 3), RD, true, true>(accn, f, v[I], ws, vo, ((t0 + I + RD) & (CH - 1)) * CSB),
            I == 0 ? publish() : void()),
           ...);
        }(std::make_integer_sequence<int, TPW>{});
      } else if constexpr (HO) {
        publish();
        [&]<int... I>(std::integer_sequence<int, I...>) {
          (w4_chunk<TPW, (I & 3), RD, true, true>(accn, f, v[I], ws, vo, ((t0 + I + RD) & (CH - 1)) * CSB), ...);
        }(std::make_integer_sequence<int, TPW>{});
      }
    });
    if constexpr (!HO) __syncthreads();
    }
    GO2PI_STAMP(P, sub, 28 + 3 * wave);
    if constexpr (HO) w4_wait<NW>(flags, wave, ep, lane, hot.err);
    GO2PI_STAMP(P, sub, 29 + 3 * wave);
    // LDS phase: the other waves' chunks, rotated order from t0 + TPW
    constexpr int K0 = HO ? TPW : 0;                             // first chunk index of the LDS phase
    constexpr int NT = (CH - K0) % 4 ? (CH - K0) % 4 : 4;       // chunks in the LDS phase's last group
    if (more) {
      w4_lds_phase<TPW, RD, (K0 & 3), NT, true>(Y, S, lane, CH, kb1, K0, ws, CSB, wn, CSB, kb1, CH, vo, accn, f);
    } else {
      load_head();  // the head's fragments, behind the last LDS phase
      w4_lds_phase<TPW, RD, (K0 & 3), NT, false>(Y, S, lane, CH, kb1, K0, ws, CSB, wn, CSB, 0, 1, vo, accn, f);
    }
    GO2PI_STAMP(P, sub, 30 + 3 * wave);
#pragma unroll
    for (int i = 0; i < TPW; ++i) {
      acc[i] = accn[i];
      bv[i] = bvn[i];
    }
    Y = Y == X0 ? Y0 : X0;
    GO2PI_STAMP(P, lane == 0 && step == 0 && l < 8, 16 + 3 * wave + (l < 3 ? l : 2));
    GO2PI_STAMP(P, lane == 0 && step == 0 && l < 8 && wave == 0, 6 + l);
  }
  // the last hidden layer's epilogue feeds the head from registers (no LDS copy).
  // Four accumulator chains per head tile, one per k-step of a chunk, so that no
  // MFMA waits on the one before it (a single chain paid the dependent-accumulator
  // latency 4 x TPW times), summed in a fixed order: (c0 + c1) + (c2 + c3).
  {
    constexpr int NCH = 4;
    f32x4 hacc[HT][NCH];
#pragma unroll
    for (int h = 0; h < HT; ++h)
#pragma unroll
      for (int c = 0; c < NCH; ++c) hacc[h][c] = f32x4{0.f, 0.f, 0.f, 0.f};
    act_dispatch<ACTC>(hot.hid_act, [&](auto act_k) {
      constexpr int ACT = decltype(act_k)::value;
#pragma unroll
      for (int i = 0; i < TPW; ++i) {
        float4 v;
        if constexpr (ACTC == 1) v = w4_epi_elu1<BIN>(acc[i], bv[i]);
        else v = w4_epi<ACT>(ap, acc[i], bv[i]);
#pragma unroll
        for (int h = 0; h < HT; ++h) {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            f32x4 &a = hacc[h][NCH == 4 ? j : (i & 1)];
            a = mfma4(f4c(hw[h][i], j), f4c(v, j), a);
          }
        }
      }
    });
#pragma unroll
    for (int h = 0; h < HT; ++h) {
      f32x4 t = hacc[h][0] + hacc[h][1];
      if constexpr (NCH == 4) t = t + (hacc[h][2] + hacc[h][3]);
      scratch[(h * NW + wave) * 64 + lane] = t;
    }
  }
  __syncthreads();
  GO2PI_STAMP(P, threadIdx.x == 0 && step == 0 && nh < 9, 6 + nh);
  if (wave < HT) {  // head tile `wave`: the four waves' partials in a fixed order, bias, final store
    f32x4 hs[1] = {scratch[(wave * NW) * 64 + lane]};
#pragma unroll
    for (int w = 1; w < NW; ++w) hs[0] += scratch[(wave * NW + w) * 64 + lane];
    GO2PI_STAMP(P, lane == 0 && wave == 0 && step == 0, 54);  // tail marks: 54 partials summed, 55 stored
    // no action post-processing (the lean kernel; a general-body program without
    // tanh / clip / scale, e.g. a GRU policy): the head's activation (usually none)
    // and the plain store of the valid rows / columns, from the hot fields
    if constexpr (!CTL && PL) {
      // the lean kernel: one store sequence; the head's activation (identity for the
      // exported policies) applied per element only when there is one. (with_act here
      // compiled the store once per activation kind: a branch ladder and the address
      // arithmetic from SGPRs spilled to VGPR lanes, ~660 cycles from the partial sums
      // to the store, profiles/r05_clock_mlp512.json tail_store.)
      const int row = row0 + (lane & 15), n0 = wave * 16 + ((lane >> 4) << 2);
      float4 v = make_float4(hs[0][0] + hbv[0].x, hs[0][1] + hbv[0].y, hs[0][2] + hbv[0].z, hs[0][3] + hbv[0].w);
      if (hot.head_act != 0) {
        v.x = act_fn(hot.head_act, hot.head_alpha, hot.head_beta, v.x);
        v.y = act_fn(hot.head_act, hot.head_alpha, hot.head_beta, v.y);
        v.z = act_fn(hot.head_act, hot.head_alpha, hot.head_beta, v.z);
        v.w = act_fn(hot.head_act, hot.head_alpha, hot.head_beta, v.w);
      }
      if (row < B) {  // (ac = the action rows of all steps, this step's at step * B rows)
        float *o = ac + ((size_t)step * B + row) * hot.head_n;
        if ((hot.head_n & 3) == 0 && ((uintptr_t)ac & 15) == 0) {  // (12 actions: one 16-byte store per lane)
          if (n0 < hot.head_n) *reinterpret_cast<float4 *>(o + n0) = v;
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (n0 + r < hot.head_n) o[n0 + r] = f4c(v, r);
        }
      }
    } else if (!CTL && hot.post_plain) {
      const int row = row0 + (lane & 15), n0 = wave * 16 + ((lane >> 4) << 2);
      with_act(hot.head_act, [&](auto act_k) {
        constexpr int ACT = decltype(act_k)::value;
        const float4 v = w4_epi<ACT>(ActP{hot.head_act, hot.head_alpha, hot.head_beta}, hs[0], hbv[0]);
        if (row < B) {  // (lean kernel: ac = the action rows of all steps, this step's at step * B
                        // rows; general body: ac = this step's rows already)
          float *o = ac + ((PL ? (size_t)step * B : (size_t)0) + row) * hot.head_n;
          if ((hot.head_n & 3) == 0 && ((uintptr_t)ac & 15) == 0) {  // (12 actions: one 16-byte store per lane)
            if (n0 < hot.head_n) *reinterpret_cast<float4 *>(o + n0) = v;
          } else {
#pragma unroll
            for (int r = 0; r < 4; ++r)
              if (n0 + r < hot.head_n) o[n0 + r] = f4c(v, r);
          }
        }
      });
    } else if constexpr (CTL && PL) {
      // the lean tick: the program's action epilogue is the identity (w4_plain) and the
      // head's fields were read with the hot block, before the tile's observation rows
      // went out. (dense_store read them here: vector loads queued behind those 6 KB of
      // row stores, so the action stores waited for all of them.)
      // (one store sequence, the head's activation per element only when there is one:
      // as the lean kernel's tail above)
      const int row = row0 + (lane & 15), n0 = wave * 16 + ((lane >> 4) << 2);
      float4 v = make_float4(hs[0][0] + hbv[0].x, hs[0][1] + hbv[0].y, hs[0][2] + hbv[0].z, hs[0][3] + hbv[0].w);
      if (hot.head_act != 0) {
        v.x = act_fn(hot.head_act, hot.head_alpha, hot.head_beta, v.x);
        v.y = act_fn(hot.head_act, hot.head_alpha, hot.head_beta, v.y);
        v.z = act_fn(hot.head_act, hot.head_alpha, hot.head_beta, v.z);
        v.w = act_fn(hot.head_act, hot.head_alpha, hot.head_beta, v.w);
      }
      if (row < B) {
        if (hot.head_n == GO2PI_CTL_DOF) {
          if (n0 < GO2PI_CTL_DOF) ctl_store4(cv, row, n0, {v.x, v.y, v.z, v.w});
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (n0 + r < hot.head_n) ctl_store(cv, row, n0 + r, f4c(v, r));
        }
      }
    } else {
      float4 none[1];
      dense_store<1>(P, P.L[nh], hs, hbv, wave, HT, lane, true, nullptr, 0, ac, cv, row0, B, none);
    }
    GO2PI_STAMP(P, lane == 0 && wave == 0 && step == 0, 55);
  }
}

// Body of the batched kernel. CTL: controller tick (steps == 1) — the
// observation is assembled from raw robot state (ctl_assemble) instead of
// read, and the final layer's store is the action post-processing (ctl_store).
// The lean pipeline kernel (policy_mlp_kernel): a dense policy whose observation
// needs no prologue arithmetic and whose action no epilogue, every hidden layer
// 64 * TPW wide with one activation, layer 0 no wider. Everything its prologue
// touches arrives as kernel arguments preloaded into SGPRs (obs, the fragment
// arena, the packed biases, the dims word): the observation, bias and layer-0
// fragment loads issue at wave start with no memory round trip in front of them
// (each dependent load at kernel start costs ~1.5K cycles: the L2s are cold), and
// the rest of the program's hot block is loaded beside them, needed only later.
// dims = in_dim | c0 << 12 | hidden layers << 20. The LDS stride is a
// compile-time constant; padding lanes of the observation tile read an element of
// the same row (times a zero weight column), rows past B the last row.
template <int TPW, int HT, int C0M, int ACTC, int NHC, int NW = 4>
__device__ __forceinline__ void w4_plain_body(const DevProgram &P, const float *__restrict__ obs,
                                              float *__restrict__ act, const float *l0w, const float *bpack, int B,
                                              int steps, unsigned dims, unsigned *yield) {
  GO2PI_ENTRY_CLOCK();
  extern __shared__ float4 lds4[];
  float *lds = reinterpret_cast<float *>(lds4);
  // tell idle resident kernels on this device to give their CUs back (resident.hip)
  if (blockIdx.x == 0 && threadIdx.x == 0 && gridDim.x > GO2PI_YIELD_MIN_GRID)
    __hip_atomic_fetch_add(yield, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const int in_dim = (int)(dims & 0xFFFu), c0 = (int)((dims >> 12) & 0xFFu), nh = (int)((dims >> 20) & 0xFFu);
  // (the program's fields are read inside w4_step once the first loads are out)
  const W4Hot hot = W4Hot{l0w, nullptr, nullptr, bpack, nullptr, nh * 16 * NW * TPW, 0, c0, 0, 0, 0.f, 0.f, 1, 0.f, 0.f};
  constexpr int S = 16 * NW * TPW + 4;  // = P.lds_stride (the engine selects this kernel only then)
  float *bufA = lds, *bufB = lds + GO2PI_TILE_ROWS * S;
  f32x4 *scratch = reinterpret_cast<f32x4 *>(lds + 2 * GO2PI_TILE_ROWS * S);
  int *flags = reinterpret_cast<int *>(lds + 2 * GO2PI_TILE_ROWS * S + 256 * NW * HT);
  float *lbias = reinterpret_cast<float *>(flags) + GO2PI_FLAG_FLOATS;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int row0 = blockIdx.x * GO2PI_TILE_ROWS;
  const int nch = (16 * c0 + 63) >> 6;  // 64-column chunks of the observation tile
  int ep = 0;                           // flag epochs published so far (the same in every wave)
  float4 ring_none[4][TPW];             // (w4_step loads its own ring here)
  for (int step = 0; step < steps; ++step) {
    // wave w stages rows w, w + NW, ... in whole 64-column chunks by direct-to-LDS
    // loads
    const float *ob = obs + (size_t)step * B * in_dim;
#pragma unroll
    for (int i = 0; i < GO2PI_TILE_ROWS / NW; ++i) {
      const int r = wave + NW * i, row = min(row0 + r, B - 1);
      const float *rp = ob + (size_t)row * in_dim;
      for (int c = 0; c < nch; ++c)
        __builtin_amdgcn_global_load_lds((gvoid_t *)(rp + min(c * 64 + lane, in_dim - 1)),
                                         (lvoid_t *)(bufA + r * S + c * 64), 4, 0, 0);
    }
    if (step == 0 && tid < NW) flags[tid] = 0;
    GO2PI_STAMP_ENTRY(P, tid == 0 && step == 0);
    GO2PI_STAMP(P, tid == 0 && step == 0, 40);
    GO2PI_STAMP(P, tid == 0 && step == 0, 41);
    w4_step<TPW, HT, false, true, C0M, ACTC, NHC, NW>(P, hot, bufA, bufB, S, scratch, flags, lbias, ep, wave, lane, act, CtlView{}, row0, B, DevCtl{},
                                       CtlLds{}, step, ring_none, false);
  }
  GO2PI_STAMP(P, tid == 0, 2);
  GO2PI_STAMP_RT(P, tid == 0, 3);
}

// The lean controller tick (r05): the controller prologue and
// epilogue (ctl_fn.hpp) around the lean pipeline, for a dense policy with the
// compile-time Elu and three hidden layers. Everything the input staging needs
// arrives as kernel arguments preloaded into SGPRs: the tile's state, joystick,
// previous observation and previous action rows and the controller parameters (q0)
// go out as direct-to-LDS loads in the first ~200 cycles, where the general body
// issued them ~2.7K cycles in, behind the chain kernel argument -> program -> its
// fields (profiles/r05_clock_ctl.json, init_subphases.obs_issued). The rest of the
// program and the controller arguments are read behind those loads.
// shape = B | in_dim << 20 (B < 2^20, in_dim < 2^12: the engine checks). c0: layer 0's
// k-chunk count (its K padded to 16 or to 64: not derivable from in_dim alone), needed
// only after the staging, from the argument segment.
template <int TPW, int HT, int C0M>
__device__ __forceinline__ void w4_ctl_body(const DevProgram &P, const DevCtl &ctl, const float *l0w,
                                            const float *bpack, unsigned shape, unsigned *yield, int c0) {
  GO2PI_ENTRY_CLOCK();
  extern __shared__ float4 lds4[];
  float *lds = reinterpret_cast<float *>(lds4);
  const int B = (int)(shape & 0xFFFFFu), in_dim = (int)(shape >> 20);
  constexpr int S = 64 * TPW + 4, NBIAS = 3 * 64 * TPW;  // (three hidden layers, NHC = 3)
  float *bufA = lds, *bufB = lds + GO2PI_TILE_ROWS * S;
  f32x4 *scratch = reinterpret_cast<f32x4 *>(lds + 2 * GO2PI_TILE_ROWS * S);
  int *flags = reinterpret_cast<int *>(lds + 2 * GO2PI_TILE_ROWS * S + 256 * 4 * HT);
  float *lbias = reinterpret_cast<float *>(flags) + GO2PI_FLAG_FLOATS;
  // (the previous observation rows in bufB: layer 0's output buffer, written only after
  // the assembly and the barrier behind it; as fused_body)
  const CtlLds CL = ctl_lds(lbias + NBIAS, GO2PI_TILE_ROWS, in_dim, bufB);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int row0 = blockIdx.x * GO2PI_TILE_ROWS;
  ctl_lds_load(CL, ctl, row0, min(GO2PI_TILE_ROWS, B - row0), in_dim, tid, wave, lane, 4);
  if (tid < 4) flags[tid] = 0;
  // tell idle resident kernels on this device to give their CUs back (resident.hip),
  // behind the staging loads
  if (blockIdx.x == 0 && tid == 0 && gridDim.x > GO2PI_YIELD_MIN_GRID)
    __hip_atomic_fetch_add(yield, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  GO2PI_STAMP_ENTRY(P, tid == 0);
  GO2PI_STAMP(P, tid == 0, 41);
  const W4Hot hot = W4Hot{l0w, nullptr, nullptr, bpack, nullptr, NBIAS, 0, c0, 0, 0, 0.f, 0.f, 1, 0.f, 0.f, in_dim};
  const CtlView cv = ctl_view(ctl, CL, row0);
  int ep = 0;
  float4 ring_none[4][TPW];  // (w4_step loads its own ring here)
  w4_step<TPW, HT, true, true, C0M, 1, 3>(P, hot, bufA, bufB, S, scratch, flags, lbias, ep, wave, lane, nullptr, cv,
                                          row0, B, ctl, CL, 0, ring_none, false);
  GO2PI_STAMP(P, tid == 0, 2);
  GO2PI_STAMP_RT(P, tid == 0, 3);
}

// The lean GRU tick (r05): a GRU cell (lbr = 1, H = 64 GT) in
// front of a dense chain the lean kernel serves (Elu, three hidden layers 64 TPW wide, no
// prologue or epilogue arithmetic). The general body's prologue was instruction-bound:
// ~1.2K scalar and spill instructions of run-time shape arithmetic between the
// observation's loads, the hidden rows' loads and the cell (clock marks 41 / 56 / 57:
// 1.7K, 3.8K, 6.2K cycles, profiles/r05_clock_gru256.json). Here the shape is compile
// time (H, the LDS stride, the bias pack), and the observation, hidden state, cell
// weights, dense arena, bias pack and B | in_dim << 20 are the preloaded kernel
// arguments, so the observation rows, the hidden rows (16-byte direct-to-LDS loads: one
// per 256 units of a row) and the cell's first fragments go out at once. Gate biases,
// the program and yield come from the argument segment.
// LSTM (r06, the lean LSTM tick): the same body around the
// four-gate cell (w4_lstm, ONNX gates i, o, f, c; gbzr = Wb + Rb per gate). A state row
// is h | c (2H floats): the h half goes to LDS as the GRU's hidden row does, and each
// lane's c units (the units of its own h' outputs) to registers, where the cell keeps
// them across every tick of the launch; both halves go back to the state rows once.
template <int TPW, int HT, int GT, bool LSTM = false>
__device__ __forceinline__ void w4_gru_body(const DevProgram &P, const float *obs, float *act, float *hidden,
                                            const float *gw, const float *l0w, const float *bpack, unsigned shape,
                                            const float *gbzr, const float *gbh, int steps, unsigned *yield) {
  GO2PI_ENTRY_CLOCK();
  extern __shared__ float4 lds4[];
  float *lds = reinterpret_cast<float *>(lds4);
  constexpr int H = 64 * GT, S = 64 * TPW + 4, NBIAS = 3 * 64 * TPW;
  constexpr int SW = LSTM ? 2 * H : H;  // state floats per robot row
  static_assert(H <= 64 * TPW, "the hidden rows fit the LDS row");
  const int B = (int)(shape & 0xFFFFFu), in_dim = (int)(shape >> 20);
  const int ipad = (in_dim + 63) & ~63, nch = ipad >> 6;  // (pack_gru: x padded to whole 64-column groups)
  float *bufA = lds, *bufB = lds + GO2PI_TILE_ROWS * S, *bufH = lds + 2 * GO2PI_TILE_ROWS * S;
  f32x4 *scratch = reinterpret_cast<f32x4 *>(lds + 3 * GO2PI_TILE_ROWS * S);
  int *flags = reinterpret_cast<int *>(lds + 3 * GO2PI_TILE_ROWS * S + 256 * 4 * HT);
  float *lbias = reinterpret_cast<float *>(flags) + GO2PI_FLAG_FLOATS;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int row0 = blockIdx.x * GO2PI_TILE_ROWS;
  // wave w stages rows w, w + 4, w + 8, w + 12; padding lanes read an element of the same
  // row (times a zero weight column), rows past B the last row (their results are dropped)
  auto stage_obs = [&](int step) {
    const float *ob = obs + (size_t)step * B * in_dim;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = wave + 4 * i;
      const float *rp = ob + (size_t)min(row0 + r, B - 1) * in_dim;
      for (int c = 0; c < nch; ++c)
        __builtin_amdgcn_global_load_lds((gvoid_t *)(rp + min(c * 64 + lane, in_dim - 1)),
                                         (lvoid_t *)(bufA + r * S + c * 64), 4, 0, 0);
    }
  };
  stage_obs(0);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = wave + 4 * i;
    const float *hp = hidden + (size_t)min(row0 + r, B - 1) * SW;
    if constexpr (H % 256 == 0) {
#pragma unroll
      for (int c = 0; c < H / 256; ++c)
        __builtin_amdgcn_global_load_lds((gvoid_t *)(hp + c * 256 + 4 * lane), (lvoid_t *)(bufH + r * S + c * 256),
                                         16, 0, 0);
    } else {
#pragma unroll
      for (int c = 0; c < H / 64; ++c)
        __builtin_amdgcn_global_load_lds((gvoid_t *)(hp + c * 64 + lane), (lvoid_t *)(bufH + r * S + c * 64), 4, 0, 0);
    }
  }
  // the dense chain's biases too: the cell's staging barrier (vmcnt behind its first
  // fragments) then covers them, so no later wait counts on the ring's loads being younger
  glds_copy(lbias, bpack, NBIAS, wave, lane, 4);
  if (tid < 4) flags[tid] = 0;
  if (blockIdx.x == 0 && tid == 0 && gridDim.x > GO2PI_YIELD_MIN_GRID)
    __hip_atomic_fetch_add(yield, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  GO2PI_STAMP_ENTRY(P, tid == 0);
  const DevGru G{gw, gbzr, gbh, in_dim, ipad, H, LSTM ? 0 : 1, LSTM ? 1 : 0, SW};
  const W4Hot hot = W4Hot{l0w, nullptr, nullptr, bpack, nullptr, NBIAS, 0, H / 16, 0, 0, 0.f, 0.f, 1, 0.f, 0.f};
  // LSTM: this lane's cell-state units, in registers for every tick (rows past B: zeros)
  float4 creg[LSTM ? GT : 1];
  if constexpr (LSTM) {
    const int row = row0 + (lane & 15);
    const float *cg = hidden + (size_t)min(row, B - 1) * SW + H + wave * GT * 16 + ((lane >> 4) << 2);
#pragma unroll
    for (int i = 0; i < GT; ++i)
      creg[i] = row < B ? *reinterpret_cast<const float4 *>(cg + i * 16) : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  int ep = 0;
  for (int step = 0; step < steps; ++step) {
    if (step > 0) stage_obs(step);
    float4 ring0[4][TPW];  // the dense chain's layer-0 ring, filled behind the cell (w4_prefill)
    float4 hn[GT];
    auto mid = [&] { w4_prefill<TPW, 0>(l0w, ring0, wave, lane); };
    if constexpr (LSTM) w4_lstm<GT>(G, bufA, bufH, bufB, S, wave, lane, hn, creg, mid);
    else w4_gru<GT>(G, bufA, bufH, bufB, S, wave, lane, hn, nullptr, mid);
    if (step == steps - 1 && row0 + (lane & 15) < B) {  // the engine's state: once, from registers
      float *hg = hidden + (size_t)(row0 + (lane & 15)) * SW + wave * GT * 16 + ((lane >> 4) << 2);
#pragma unroll
      for (int i = 0; i < GT; ++i) *reinterpret_cast<float4 *>(hg + i * 16) = hn[i];
      if constexpr (LSTM) {
#pragma unroll
        for (int i = 0; i < GT; ++i) *reinterpret_cast<float4 *>(hg + H + i * 16) = creg[i];
      }
    }
    lds_barrier();  // every wave has read bufH (an LDS hand-off: no wait for the ring's loads)
    float *hl = bufH + (lane & 15) * S + wave * GT * 16 + ((lane >> 4) << 2);
#pragma unroll
    for (int i = 0; i < GT; ++i) *reinterpret_cast<float4 *>(hl + i * 16) = hn[i];
    w4_step<TPW, HT, false, true, 0, 1, 3>(P, hot, bufB, bufA, S, scratch, flags, lbias, ep, wave, lane, act,
                                           CtlView{}, row0, B, DevCtl{}, CtlLds{}, step, ring0, true);
  }
  GO2PI_STAMP(P, tid == 0, 2);
  GO2PI_STAMP_RT(P, tid == 0, 3);
}

// RNN: the recurrent cell this instantiation runs when the program has one (0 GRU,
// 1 LSTM; one kernel per cell keeps the other cell's registers out of it).
template <int NW, bool CTL, int W4T = 0, int W4H = 0, int C0M = 0, int RNN = 0, int ACTC = -1, int NHC = 0>
__device__ __forceinline__ void fused_body(const DevProgram &P, const float *__restrict__ obs,
                                           float *__restrict__ act, float *__restrict__ hidden, int B, int steps,
                                           const DevCtl ctl) {
  GO2PI_ENTRY_CLOCK();
  extern __shared__ float4 lds4[];
  float *lds = reinterpret_cast<float *>(lds4);
  const int S = P.lds_stride;
  float *bufA = lds;
  float *bufB = lds + GO2PI_TILE_ROWS * S;
  float *bufH = lds + 2 * GO2PI_TILE_ROWS * S;  // only with a GRU
  f32x4 *scratch = reinterpret_cast<f32x4 *>(lds + (2 + P.has_gru) * GO2PI_TILE_ROWS * S);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int row0 = blockIdx.x * GO2PI_TILE_ROWS;
  constexpr int NT = NW * 64;
  // tell idle resident kernels on this device to give their CUs back (resident.hip)
  if (blockIdx.x == 0 && tid == 0 && P.yield && gridDim.x > GO2PI_YIELD_MIN_GRID)
    __hip_atomic_fetch_add(P.yield, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const int H = P.gru.H, SW = P.gru.sw;  // hidden width; state floats per robot (LSTM: h | c)
  // (r05) the program fields read between the first direct-to-LDS load and the recurrent
  // cell's contraction, read once here, before any. The compiler models a direct-to-LDS
  // load as a store to memory, so a program field read after one waited vmcnt(0), the
  // staging loads' whole HBM round trip, each time: GRU-256 tick, observation loads
  // issued at 1.9K cycles, hidden rows at 3.9K, the cell entered at 6.6K
  // (profiles/r05_clock_gru256.json, slots 41, 56, 58)
  const int zero_fill = P.zero_fill, has_gru = P.has_gru, out_dim = P.out_dim, in_dim0 = P.in_dim,
            in_pad0 = P.in_pad;
  const float *pzero = P.zero;
  const DevGru G = P.gru;
  const float *w4_bpack = P.w4_bpack, *l0_w = P.l0_w;
  const int w4_bias = P.w4_bias;
  // (clock builds: this workgroup's stamp row, read here too, so that the prologue's
  // marks do not wait for the staging loads themselves)
#ifdef GO2PI_DIAG_CLOCK
  unsigned long long *srow = P.stamps ? P.stamps + blockIdx.x * GO2PI_STAMPS_PER_WG : nullptr;
#else
  unsigned long long *srow = nullptr;
#endif
  (void)srow;
  // Touch every layer descriptor up front: one burst of scalar loads warms the
  // scalar cache, so each layer's start does not pay a K$ miss on its fields
  // (measured: layer entry ~990 -> ~740 cycles after the barrier).
  if constexpr (W4T > 0) {
    // pipeline: no warm-up (holding every descriptor in SGPRs spilled them to VGPR
    // lanes; the fields are read where needed and hit the scalar cache after the
    // first layer)
  } else {
    int d = 0;
    for (int l = 0; l < P.nl; ++l) d ^= P.L[l].K_pad ^ P.L[l].N_pad ^ P.L[l].act ^ (int)(size_t)P.L[l].w;
    asm volatile("" ::"s"(d));  // consumes the loads; no side effect
  }
  // init sub-phases: 40 descriptors warm, 41 observation loads issued, 42 pipeline barrier reached
  GO2PI_STAMP(P, tid == 0, 40);
  GO2PI_STAMP_ENTRY(P, tid == 0);

  // controller tick: this tile's raw inputs staged in LDS behind the scratch
  // region (one burst of direct-to-LDS loads), then assembled from there
  // per-wave layer hand-off flags (Handoff) behind the scratch region, cleared
  // here; every path passes a workgroup barrier before the first layer
  float *after_scratch = lds + (2 + P.has_gru) * GO2PI_TILE_ROWS * S + 256 * NW * (P.head_fuse > 1 ? P.head_fuse : 1);
  int *flags = reinterpret_cast<int *>(after_scratch);
  if (tid < NW) flags[tid] = 0;
  int ep = 0;  // hand-offs published so far (identical in every wave)
  // (the pipeline's bias copy sits between the flags and the controller-tick region)
  float *lbias = after_scratch + GO2PI_FLAG_FLOATS;
  // (the previous observation rows in bufB: layer 0's output buffer, written only after
  // the assembly and the barrier behind it)
  const CtlLds CL = ctl_lds(lbias + P.w4_bias, GO2PI_TILE_ROWS, P.in_dim, bufB);
  CtlView cv{};
  CtlQ cq{};
  // the pipeline without a recurrent cell assembles the tick's observation inside
  // w4_step, behind layer 0's first fragment loads (their latency and the raw rows'
  // overlap); every other body assembles it here, before anything else
  const bool ctl_late = CTL && W4T > 0 && !P.has_gru;
  if constexpr (CTL) {
    cq = ctl_q(P, ctl);
    cv = ctl_view(ctl, CL, row0);
    ctl_lds_load(CL, ctl, row0, min(GO2PI_TILE_ROWS, B - row0), P.in_dim, tid, wave, lane, NW);
    if (!ctl_late) {
      lds_dma_wait();
      __syncthreads();
    }
    GO2PI_STAMP(P, tid == 0 && !ctl_late, 5);
  }
  // plain observation rows with no prologue arithmetic are staged by direct-to-LDS
  // loads (needs whole 64-column chunks to fit the LDS row)
  const bool glds_obs = !CTL && !P.pre_sub && !P.pre_div && !P.pre_mul && !P.pre_clip && ((P.in_pad + 63) & ~63) <= S;
  auto stage_obs = [&](int step) {
    if constexpr (CTL) {  // this tile's rows of ctl.obs are read only from the LDS image: publish in place
      if (ctl_late) return;  // (w4_step)
      ctl_assemble_flat<true>(P, CL, cq, ctl.joy != nullptr, min(GO2PI_TILE_ROWS, B - row0), bufA, S,
                              ctl.obs + (size_t)row0 * P.in_dim, tid, NT);
    } else if (W4T > 0 && glds_obs) {
      // pipeline: wave w stages rows w, w + 4, w + 8, w + 12 in whole 64-column
      // chunks (in_pad is a GRU's input width, not always a multiple of 64);
      // per-lane source pointers are formed once, so the loop carries no scalar
      // reloads between the direct-to-LDS loads
      const int in_dim = in_dim0, nch = (in_pad0 + 63) >> 6;
      const float *ob = obs + (size_t)step * B * in_dim;
      const float *zero = pzero + lane;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = wave + 4 * i, row = row0 + r;
        const float *rp = ob + (size_t)row * in_dim + lane;
        for (int c = 0; c < nch; ++c) {
          const float *src = (row < B && c * 64 + lane < in_dim) ? rp + c * 64 : zero;
          __builtin_amdgcn_global_load_lds((gvoid_t *)src, (lvoid_t *)(bufA + r * S + c * 64), 4, 0, 0);
        }
      }
    } else if (glds_obs) {
      // one direct-to-LDS load per (row, 64-column chunk): the tile's observation
      // loads all in flight together; padding lanes and rows past B read zeros
      const float *ob = obs + (size_t)step * B * P.in_dim;
      const int nch = (P.in_pad + 63) >> 6;
      for (int jb = wave; jb < GO2PI_TILE_ROWS * nch; jb += NW) {
        const int r = jb / nch, c = jb - r * nch, row = row0 + r, k = c * 64 + lane;
        const float *src = (row < B && k < P.in_dim) ? ob + (size_t)row * P.in_dim + k : P.zero + lane;
        __builtin_amdgcn_global_load_lds((gvoid_t *)src, (lvoid_t *)(bufA + r * S + c * 64), 4, 0, 0);
      }
    } else {
      const float *ob = obs + (size_t)step * B * P.in_dim;
      for (int e = tid; e < GO2PI_TILE_ROWS * P.in_pad; e += NT) {
        const int r = e / P.in_pad, k = e - r * P.in_pad, row = row0 + r;
        float v = 0.f;
        if (row < B && k < P.in_dim) v = prologue(P, ob[(size_t)row * P.in_dim + k], k);
        bufA[r * S + k] = v;
      }
    }
  };
  // Step 0's observation loads go out first; their HBM latency overlaps the
  // zero fill. Padded activation columns are read (against zero weights) by the
  // next layer, so they must hold finite values: clear everything the
  // observation does not cover, once.
  stage_obs(0);
  GO2PI_STAMP_AT(srow, tid == 0, 41);
  if (zero_fill) {  // only a GRU whose H is not a multiple of 64 leaves such columns
    const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
    const int tail4 = (S - in_pad0) >> 2;
    for (int e = tid; e < GO2PI_TILE_ROWS * tail4; e += NT) {
      const int r = e / tail4;
      reinterpret_cast<float4 *>(bufA + r * S + in_pad0)[e - r * tail4] = z;
    }
    if constexpr (CTL) __syncthreads();  // every wave done reading the previous observation rows in bufB
    float4 *l4 = reinterpret_cast<float4 *>(bufB);
    const int n4 = ((1 + has_gru) * GO2PI_TILE_ROWS * S) >> 2;
    for (int e = tid; e < n4; e += NT) l4[e] = z;
  }
  if (has_gru) {
    // the zero fill above before the hidden rows land (otherwise no barrier: the
    // hidden rows' direct-to-LDS loads go out beside the observation's)
    if (zero_fill) __syncthreads();
    if (W4T > 0 && H % 64 == 0) {
      // pipeline: the hidden rows by direct-to-LDS loads, in flight with the
      // observation's (one 64-column chunk per instruction; rows past B read zeros)
      for (int i = 0; i < 4; ++i) {
        const int r = wave + 4 * i, row = row0 + r;
        for (int c = 0; c < (H >> 6); ++c) {
          const float *src = row < B ? hidden + (size_t)row * SW + c * 64 + lane : pzero + lane;
          __builtin_amdgcn_global_load_lds((gvoid_t *)src, (lvoid_t *)(bufH + r * S + c * 64), 4, 0, 0);
        }
      }
    } else {
      for (int e = tid; e < GO2PI_TILE_ROWS * H; e += NT) {
        const int r = e / H, k = e - r * H, row = row0 + r;
        bufH[r * S + k] = row < B ? hidden[(size_t)row * SW + k] : 0.f;
      }
    }
  }
  GO2PI_STAMP_AT(srow, tid == 0 && has_gru, 56);  // (GRU prologue marks: 56 hidden rows issued, 57 step loop, 58 cell entry)
  // LSTM, pipeline: this lane's cell-state units (w4_lstm) in registers for the whole sequence
  float4 creg[4];
  if (RNN == 1 && W4T > 0 && has_gru && (H == 256 || H == 128)) {
    const int GT = H >> 6, row = row0 + (lane & 15);
    const float *cg = hidden + (size_t)row * SW + H + wave * GT * 16 + ((lane >> 4) << 2);
#pragma unroll
    for (int i = 0; i < 4; ++i)
      creg[i] = (i < GT && row < B) ? *reinterpret_cast<const float4 *>(cg + i * 16) : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  for (int step = 0; step < steps; ++step) {
    float *ac = act + (size_t)step * B * out_dim;
    GO2PI_STAMP_AT(srow, tid == 0 && step == 0 && has_gru, 57);
    if (step > 0) stage_obs(step);
    if constexpr (W4T > 0) {  // the 4-wave uniform-MLP pipeline (its own barriers)
      static_assert(NW == 4, "one wave per SIMD");
      float *X0 = bufA, *Y0 = bufB;
      float4 ring0[4][W4T > 0 ? W4T : 1];  // layer 0's ring, filled behind a recurrent cell (w4_prefill)
      bool ring_pre = false;
      if (has_gru) {  // recurrent policy: the GRU cell first, h' is the pipeline's input
        // the pipelined cell (w4_gru / w4_lstm wait for the x / h staging and barrier
        // themselves): h' to bufB, registers, and the carry
        auto carry = [&](auto gt_k) {
          constexpr int GT = decltype(gt_k)::value;
          float4 hn[GT];
          constexpr bool lstm = RNN == 1;
          // layer 0's first fragments (and, on the first step, the hidden layers' biases)
          // go out between the cell's contraction and its gate math: their L2 / HBM
          // latency overlaps the epilogue and the hidden-row carry instead of
          // following them (w4_step then starts from this ring)
          // (not in the LSTM body with a run-time activation: its ring registers spilled)
          constexpr bool PREF = !(lstm && ACTC != 1);
          auto mid = [&] {
            if constexpr (PREF) {
              if (step == 0) glds_copy(lbias, w4_bpack, w4_bias, wave, lane, 4);
              w4_prefill<W4T, C0M>(l0_w, ring0, wave, lane);
            }
          };
          GO2PI_STAMP_AT(srow, tid == 0 && step == 0, 58);
          if constexpr (lstm) {
            float4 cr[GT];
#pragma unroll
            for (int i = 0; i < GT; ++i) cr[i] = creg[i];
            w4_lstm<GT>(G, bufA, bufH, bufB, S, wave, lane, hn, cr, mid);
#pragma unroll
            for (int i = 0; i < GT; ++i) creg[i] = cr[i];
          } else {
            w4_gru<GT>(G, bufA, bufH, bufB, S, wave, lane, hn,
                       step == 0 ? srow : nullptr, mid);
          }
          ring_pre = PREF;
          if (step == steps - 1 && row0 + (lane & 15) < B) {  // the engine's state: once, from registers
            float *hg = hidden + (size_t)(row0 + (lane & 15)) * SW + wave * GT * 16 + ((lane >> 4) << 2);
#pragma unroll
            for (int i = 0; i < GT; ++i) *reinterpret_cast<float4 *>(hg + i * 16) = hn[i];
            if constexpr (lstm) {
#pragma unroll
              for (int i = 0; i < GT; ++i) *reinterpret_cast<float4 *>(hg + H + i * 16) = creg[i];
            }
          }
          __syncthreads();  // every wave has read bufH
          float *hl = bufH + (lane & 15) * S + wave * GT * 16 + ((lane >> 4) << 2);
#pragma unroll
          for (int i = 0; i < GT; ++i) *reinterpret_cast<float4 *>(hl + i * 16) = hn[i];
        };
        if (H == 256) {
          carry(std::integral_constant<int, 4>{});
        } else if (H == 128) {
          carry(std::integral_constant<int, 2>{});
        } else {
          lds_dma_wait();
          __syncthreads();  // x in bufA, the hidden rows in bufH
          if constexpr (RNN == 1) lstm_cell<NW>(P.gru, bufA, bufH, bufB, S, wave, lane, hidden, row0, B);
          else gru_cell<NW>(P.gru, bufA, bufH, bufB, S, wave, lane);
          __syncthreads();
          for (int e = tid; e < GO2PI_TILE_ROWS * H; e += NT) {
            const int r = e / H, k = e - r * H;
            bufH[r * S + k] = bufB[r * S + k];  // read again only in the next step, after w4_step's barriers
          }
        }
        X0 = bufB;
        Y0 = bufA;
      }
      w4_step<W4T, W4H, CTL, false, C0M, ACTC, NHC>(P, w4_hot(P), X0, Y0, S, scratch, flags, lbias, ep, wave, lane, ac,
                                                    cv, row0, B, ctl, CL, step, ring0, ring_pre);
      continue;
    }
    lds_dma_wait();  // the observation tile's direct-to-LDS loads
    __syncthreads();
    GO2PI_STAMP(P, tid == 0 && step == 0, 4);
    if constexpr (CTL) {
      if (ctl.status && tid < min(GO2PI_TILE_ROWS, B - row0)) ctl.status[row0 + tid] = CL.nanf[tid];
      GO2PI_STAMP(P, tid == 0, 15);
    }
    float *X = bufA, *Y = bufB;
    if (P.has_gru) {
      if constexpr (RNN == 1) lstm_cell<NW>(P.gru, bufA, bufH, bufB, S, wave, lane, hidden, row0, B);
      else gru_cell<NW>(P.gru, bufA, bufH, bufB, S, wave, lane);
      __syncthreads();
      for (int e = tid; e < GO2PI_TILE_ROWS * H; e += NT) {
        const int r = e / H, k = e - r * H;
        bufH[r * S + k] = bufB[r * S + k];
      }
      X = bufB;
      Y = bufA;
      // no barrier needed: layer 0 below reads bufB (X) and writes bufA (Y); bufH is
      // next read after the end-of-step barrier
    }
    for (int l = 0; l < P.nl; ++l) {
      const bool last = l == P.nl - 1;
      if (P.head_fuse && l == P.nl - 2) {
        if (P.head_fuse == 1)
          dense_layer_head<NW, 1>(P, P.L[l], P.L[l + 1], X, Y, S, scratch, wave, lane, row0, B);
        else dense_layer_head<NW, 2>(P, P.L[l], P.L[l + 1], X, Y, S, scratch, wave, lane, row0, B);
        __syncthreads();
        head_finish<NW>(P, P.L[l + 1], scratch, wave, lane, ac, cv, row0, B);
        // slots 6..14 (15 is the controller tick's)
        GO2PI_STAMP(P, tid == 0 && step == 0 && l < 8, 6 + l);
        GO2PI_STAMP(P, tid == 0 && step == 0 && l < 8, 7 + l);
        break;  // scratch is next written two barriers later; bufA/bufB are free
      }
      dense_layer<NW>(P, P.L[l], X, Y, S, scratch, wave, lane, last, ac, cv, row0, B);
      __syncthreads();  // a workgroup barrier after every layer (dense_acc: flags measured slower)
      GO2PI_STAMP(P, tid == 0 && step == 0 && l < 9, 6 + l);  // slots 6..14 (15 is the controller tick's)
      float *t = X;
      X = Y;
      Y = t;
    }
  }
  if (P.has_gru && !(W4T > 0 && (H == 256 || H == 128))) {  // (the pipelined cells store it from registers)
    for (int e = tid; e < GO2PI_TILE_ROWS * H; e += NT) {
      const int r = e / H, k = e - r * H, row = row0 + r;
      if (row < B) hidden[(size_t)row * SW + k] = bufH[r * S + k];
    }
  }
  GO2PI_STAMP(P, tid == 0, 2);
  GO2PI_STAMP_RT(P, tid == 0, 3);
}

// W4T > 0: the 4-wave uniform-MLP pipeline with W4T tiles per wave and a W4H-tile
// head (one kernel per shape: a single pipeline per kernel keeps the program
// argument in SGPRs and the ring in registers)
// The program is read from its device-memory copy (L2-resident across launches)
// rather than passed by value: a by-value kernarg is a fresh copy per launch, and
// every cache line of it a workgroup first touches is a memory round trip.
inline size_t fused_ctl_lds_bytes(const DevProgram &p, int waves) {
  return fused_lds_bytes(p, waves) + sizeof(float) * ctl_lds_floats(GO2PI_TILE_ROWS, p.in_dim, false);
}

// The 4-wave pipeline's host side, one translation unit per tiles per wave
// (kernels_w4_t{2,4,8}.hip; each picks the head width, lean / general body and
// layer-0 chunk shape from the program).
template <int TPW>
int w4_configure(const DevProgram &p);
template <int TPW>
int w4_launch(const DevProgram &p, const DevProgram *p_dev, const float *obs, float *act, float *hidden, int batch,
              int steps, void *stream);
template <int TPW>
int w4_launch_ctl(const DevProgram &p, const DevProgram *p_dev, const DevCtl &ctl, float *hidden, int batch,
                  void *stream);
// The generic body's host side, one translation unit per wave count
// (kernels_gen_w{4,8,16}.hip).
template <int NW>
int gen_configure(const DevProgram &p);
template <int NW>
int gen_launch(const DevProgram &p, const DevProgram *p_dev, const float *obs, float *act, float *hidden, int batch,
               int steps, void *stream);
template <int NW>
int gen_launch_ctl(const DevProgram &p, const DevProgram *p_dev, const DevCtl &ctl, float *hidden, int batch,
                   void *stream);

template <int NW, int W4T = 0, int W4H = 0, int C0M = 0, int RNN = 0, int ACTC = -1, int NHC = 0>
__global__ __launch_bounds__(NW * 64) void policy_fused_kernel(const DevProgram *__restrict__ Pd,
                                                               const float *__restrict__ obs,
                                                               float *__restrict__ act, float *__restrict__ hidden,
                                                               int B, int steps) {
  fused_body<NW, false, W4T, W4H, C0M, RNN, ACTC, NHC>(*Pd, obs, act, hidden, B, steps, DevCtl{});
}

// The lean pipeline kernel (w4_plain_body). Argument order = preload order: the
// first 16 dwords of the kernel arguments arrive in SGPRs (kernels_w4_t*.hip are
// built with -amdgpu-kernarg-preload-count=16); these are 13.
// NW: waves per workgroup, 4 (one per SIMD, the r01-r04 pipeline) or 8 (two per SIMD,
// TPW tiles each: while one wave of a SIMD runs its epilogue, the other's MFMAs keep
// the matrix pipe busy; tools/mfma_2wave.hip: a partner wave's epilogue VALU leaves
// the MFMA wave's 32 cycles per v_mfma_f32_16x16x4_f32 untouched, r05).
template <int TPW, int HT, int C0M, int ACTC, int NHC, int NW = 4>
__global__ __launch_bounds__(NW * 64) void policy_mlp_kernel(const float *__restrict__ obs, float *__restrict__ act,
                                                             const float *__restrict__ l0w,
                                                             const float *__restrict__ bpack,
                                                             const DevProgram *__restrict__ Pd, int B, int steps,
                                                             unsigned dims, unsigned *yield) {
  w4_plain_body<TPW, HT, C0M, ACTC, NHC, NW>(*Pd, obs, act, l0w, bpack, B, steps, dims, yield);
}

// The lean GRU tick (w4_gru_body): the arguments up to shape are preloaded into SGPRs
// (13 dwords); the rest come from the argument segment.
template <int TPW, int HT, int GT>
__global__ __launch_bounds__(256) void policy_gru_kernel(const float *__restrict__ obs, float *__restrict__ act,
                                                         float *__restrict__ hidden, const float *__restrict__ gw,
                                                         const float *__restrict__ l0w,
                                                         const float *__restrict__ bpack, unsigned shape,
                                                         const float *gbzr, const float *gbh,
                                                         const DevProgram *__restrict__ Pd, int steps,
                                                         unsigned *yield) {
  w4_gru_body<TPW, HT, GT>(*Pd, obs, act, hidden, gw, l0w, bpack, shape, gbzr, gbh, steps, yield);
}

// The lean LSTM tick (w4_gru_body's LSTM form, r06): the same arguments (gbh unused).
template <int TPW, int HT, int GT>
__global__ __launch_bounds__(256) void policy_lstm_kernel(const float *__restrict__ obs, float *__restrict__ act,
                                                          float *__restrict__ hidden, const float *__restrict__ gw,
                                                          const float *__restrict__ l0w,
                                                          const float *__restrict__ bpack, unsigned shape,
                                                          const float *gbzr, const float *gbh,
                                                          const DevProgram *__restrict__ Pd, int steps,
                                                          unsigned *yield) {
  w4_gru_body<TPW, HT, GT, true>(*Pd, obs, act, hidden, gw, l0w, bpack, shape, gbzr, gbh, steps, yield);
}

template <int NW, int W4T = 0, int W4H = 0, int C0M = 0, int RNN = 0>
__global__ __launch_bounds__(NW * 64) void policy_fused_ctl_kernel(const DevProgram *__restrict__ Pd, DevCtl C,
                                                                   float *__restrict__ hidden, int B) {
  fused_body<NW, true, W4T, W4H, C0M, RNN>(*Pd, nullptr, nullptr, hidden, B, 1, C);
}

// The lean controller tick (w4_ctl_body). The first arguments, up to shape, are
// preloaded into SGPRs (13 dwords); C (its row pointers repeat the preloaded ones),
// Pd, yield and c0 come from the kernel argument segment, needed only later.
template <int TPW, int HT, int C0M>
__global__ __launch_bounds__(256) void policy_mlp_ctl_kernel(const float *__restrict__ state,
                                                             const float *__restrict__ joy, float *__restrict__ obs,
                                                             float *__restrict__ act, const DevCtlParams *prm,
                                                             const float *__restrict__ l0w, unsigned shape,
                                                             const float *__restrict__ bpack,
                                                             const DevProgram *__restrict__ Pd, unsigned *yield,
                                                             int c0, DevCtl C) {
  DevCtl c = C;
  c.state = state;
  c.joy = joy;
  c.obs = obs;
  c.action = act;
  c.prm = prm;
  w4_ctl_body<TPW, HT, C0M>(*Pd, c, l0w, bpack, shape, yield, c0);
}

}  // namespace go2pi
