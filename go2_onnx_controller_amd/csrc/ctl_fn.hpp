// Controller-tick device helpers shared by kernels.hip and resident.hip:
// observation assembly (controller.cpp:173-212) and action post-processing
// (controller.cpp:217-223, 240-248), plus the direct-to-LDS copy they use.
#pragma once
#include <hip/hip_runtime.h>

#include "device_fn.hpp"
#include "program.hpp"

namespace go2pi {

// ---------------------------------------------------------------------------
// Controller tick. The observation is the concatenation
// of seven history blocks (controller.cpp:210-212); block b holds kHistory
// copies of a d_b-wide signal, oldest first, and each tick shifts it left by
// d_b and appends the current value (populate_buffer, controller.hpp:45-52).
// Blocks: gravity_b 3, base_ang_vel 3, vel_cmd 3, q - q0 12, dq 12, previous
// action 12, foot contacts 4 (49 per step).

// gravity_b = quaternion_.inverse() * gravity_w_ (controller.cpp:182-184) with
// Eigen 3.4 semantics: inverse() = conjugate / squaredNorm (the zero quaternion
// if squaredNorm <= 0), squaredNorm summed as (x²+z²)+(y²+w²) (SSE predux of
// the (x,y,z,w) coefficients), and q * v = _transformVector:
// uv = 2 (q.vec × v), r = (v + w uv) + q.vec × uv. Every operation rounds to
// fp32 in that order (no fma contraction), like the reference's x86 build.
// Four lanes of a quad per robot: lane i of the quad divides one
// quaternion coefficient (i = 0: w, 1: -x, 2: -y, 3: -z, over the same n2) and takes
// the other three quotients from its neighbours (DPP quad broadcasts), then forms
// component i (< 3) branch-free: one IEEE division per lane instead of four (the
// batch-1 resident kernel's assembly waits for this block: ~1.4K cycles with all four
// divisions and a branch per component in every lane). All four lanes of the quad active.
__device__ __forceinline__ float quad_bcast(float v, int k) {
  const int b = __float_as_int(v);
  switch (k) {  // quad_perm [k, k, k, k]
    case 0: return __int_as_float(__builtin_amdgcn_update_dpp(0, b, 0x00, 0xF, 0xF, false));
    case 1: return __int_as_float(__builtin_amdgcn_update_dpp(0, b, 0x55, 0xF, 0xF, false));
    case 2: return __int_as_float(__builtin_amdgcn_update_dpp(0, b, 0xAA, 0xF, 0xF, false));
    default: return __int_as_float(__builtin_amdgcn_update_dpp(0, b, 0xFF, 0xF, 0xF, false));
  }
}
__device__ __forceinline__ float ctl_gravity_quad(const float *st, float v0, float v1, float v2, int i) {
#pragma clang fp contract(off)
  const float w = st[0], x = st[1], y = st[2], z = st[3];
  const float n2 = (x * x + z * z) + (y * y + w * w);
  const float num = i == 0 ? w : (i == 1 ? -x : (i == 2 ? -y : -z));
  const float qi = n2 > 0.f ? num / n2 : 0.f;
  const float qw = quad_bcast(qi, 0), qx = quad_bcast(qi, 1), qy = quad_bcast(qi, 2), qz = quad_bcast(qi, 3);
  float u0 = qy * v2 - qz * v1, u1 = qz * v0 - qx * v2, u2 = qx * v1 - qy * v0;
  u0 += u0;
  u1 += u1;
  u2 += u2;
  const float c0 = qy * u2 - qz * u1, c1 = qz * u0 - qx * u2, c2 = qx * u1 - qy * u0;
  const float r0 = (v0 + qw * u0) + c0, r1 = (v1 + qw * u1) + c1, r2 = (v2 + qw * u2) + c2;
  return i == 0 ? r0 : (i == 1 ? r1 : r2);
}

// Direct-to-LDS copy of n contiguous floats (global_load_lds_dword: no VGPR
// round trip, every load of the workgroup in flight at once). dst needs room
// for ceil64(n) floats (the tail lanes re-read element n-1). Complete after
// the next __syncthreads() (its fence waits vmcnt(0)).
typedef __attribute__((address_space(1))) void gvoid_t;
typedef __attribute__((address_space(1))) unsigned long long gu64_t;  // (a global, not flat, access)
typedef __attribute__((address_space(3))) void lvoid_t;
// Before the barrier that hands LDS-DMA'd bytes to OTHER waves, each issuing wave
// waits for its own direct-to-LDS loads: the compiler's barrier fence does not
// count them (MI355X_MICROARCH.md §Two waves per SIMD, item 7: nothing orders a
// ds_read behind a pending LDS-DMA except the issuing wave's covering vmcnt).
__device__ __forceinline__ void lds_dma_wait() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
// Workgroup barrier that leaves this wave's N youngest vector-memory ops in flight
// (weight fragments prefetched for after the barrier); __syncthreads()'s fence
// would wait for all of them. Everything older — the LDS-DMA the barrier publishes
// — has landed: loads return in issue order. The caller keeps exactly N loads
// between the DMA and this barrier (compiler barriers on both sides).
template <int N>
__device__ __forceinline__ void wg_barrier_vm() {
  static_assert(N >= 0 && N <= 63, "vmcnt immediate");
  asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(N) : "memory");
}

// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS ops, not for
// its vector-memory ops. __syncthreads()'s fence also waits vmcnt(0), i.e. for
// weight fragments just prefetched into registers (an L2 round trip on the
// critical path of a batch-1 request's every layer) and for granule stores in flight.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

__device__ __forceinline__ void glds_copy(float *dst, const float *src, int n, int wave, int lane, int nw) {
  for (int base = wave * 64; base < n; base += nw * 64) {
    const int i = min(base + lane, n - 1);
    __builtin_amdgcn_global_load_lds((gvoid_t *)(src + i), (lvoid_t *)(dst + base), 4, 0, 0);
  }
}

// LDS image of one tile's controller inputs (rows r < R of the tile): q0
// (double), raw state rows, joystick rows, previous action / observation rows,
// per-row NaN flags. Plain values passed by value (no address-taken locals:
// nothing spills to scratch).
struct CtlLds {
  double *q0;
  float *st, *jy, *act, *obs;
  unsigned *nanf;
};

// obs: the previous observation rows get a region of their own (false: the caller
// places them, e.g. the batched kernel in its layer-0 output buffer, unused until the
// assembly is done — at a 16-step history the rows are 50 KB per tile)
__host__ __device__ inline int ctl_lds_floats(int R, int in_dim, bool obs = true) {
  auto c64 = [](int x) { return (x + 63) & ~63; };
  // q0: 12 doubles, copied by one direct-to-LDS instruction (64 lanes x 4 B: 64 floats of room)
  return 64 + c64(R * GO2PI_CTL_STATE_DIM) + c64(R * GO2PI_CTL_JOY_DIM) + c64(R * GO2PI_CTL_DOF) +
         (obs ? c64(R * in_dim) : 0) + GO2PI_TILE_ROWS;
}

__device__ __forceinline__ CtlLds ctl_lds(float *base, int R, int in_dim, float *obs = nullptr) {
  auto c64 = [](int x) { return (x + 63) & ~63; };
  CtlLds L;
  L.q0 = reinterpret_cast<double *>(base);
  L.st = base + 64;
  L.jy = L.st + c64(R * GO2PI_CTL_STATE_DIM);
  L.act = L.jy + c64(R * GO2PI_CTL_JOY_DIM);
  float *end = L.act + c64(R * GO2PI_CTL_DOF);
  L.obs = obs ? obs : end;
  L.nanf = reinterpret_cast<unsigned *>(obs ? end : end + c64(R * in_dim));
  return L;
}

// Issue the direct-to-LDS loads of rows [row0, row0 + nrows) and of q0, and clear
// the NaN flags. Nothing here waits for memory: the loads land by the issuing
// waves' next vmcnt wait (lds_dma_wait, or the pipeline's wg_barrier_vm).
__device__ __forceinline__ void ctl_lds_load(const CtlLds L, const DevCtl C, int row0, int nrows, int in_dim, int tid,
                                             int wave, int lane, int nw) {
  glds_copy(reinterpret_cast<float *>(L.q0), reinterpret_cast<const float *>(C.prm->q0), 2 * GO2PI_CTL_DOF, wave, lane,
            nw);
  glds_copy(L.st, C.state + (size_t)row0 * GO2PI_CTL_STATE_DIM, nrows * GO2PI_CTL_STATE_DIM, wave, lane, nw);
  if (C.joy) glds_copy(L.jy, C.joy + (size_t)row0 * GO2PI_CTL_JOY_DIM, nrows * GO2PI_CTL_JOY_DIM, wave, lane, nw);
  glds_copy(L.act, C.action + (size_t)row0 * GO2PI_CTL_DOF, nrows * GO2PI_CTL_DOF, wave, lane, nw);
  glds_copy(L.obs, C.obs + (size_t)row0 * in_dim, nrows * in_dim, wave, lane, nw);
  if (tid < GO2PI_TILE_ROWS) L.nanf[tid] = 0u;
}

// Controller parameters and program fields the assembly reads, loaded once (by
// value: their scalar loads overlap the input staging instead of following it, and
// none is reloaded after the assembly's stores: measured 8.6K cycles per 16-robot
// tile when the program's fields were re-read per element).
struct CtlQ {
  int hist;
  float thr, g0, g1, g2;
  int in_dim, in_pad;
  Pro pro;
};

// The controller parameters are read through the constant address space: scalar
// loads (lgkmcnt). Read through the generic pointer after the kernel's first store
// they were vector loads, and the vmcnt(0) in front of their use also waited for the
// weight fragments the pipeline keeps in flight across the input staging.
typedef const __attribute__((address_space(4))) DevCtlParams kparams_t;

__device__ __forceinline__ CtlQ ctl_q(const DevProgram &P, const DevCtl C) {
  kparams_t &Q = *(kparams_t *)C.prm;
  return CtlQ{Q.hist, Q.contact_threshold, Q.gravity_w[0], Q.gravity_w[1], Q.gravity_w[2], P.in_dim, P.in_pad,
              pro_of(P)};
}

// The lean tick's CtlQ (w4_ctl_body): a program with no observation prologue, so no
// program field is read. A program field read after the tile's direct-to-LDS loads is
// a vector load queued behind them (the loads are modelled as stores), and its wait
// would be a wait for every one of them.
__device__ __forceinline__ CtlQ ctl_q_plain(const DevCtl C, int in_dim, int in_pad) {
  kparams_t &Q = *(kparams_t *)C.prm;
  return CtlQ{Q.hist, Q.contact_threshold, Q.gravity_w[0], Q.gravity_w[1], Q.gravity_w[2], in_dim, in_pad, Pro{}};
}

// Block b of the 49 values a tick appends per robot (controller.cpp:210-212):
// 0 gravity_b 3, 1 base_ang_vel 3, 2 vel_cmd 3, 3 q - q0 12, 4 dq 12, 5 action 12,
// 6 contacts 4. cum: the block's first value among the 49; d: its width. In the
// observation row block b spans [H * cum, H * (cum + d)), the newest d values last.
__device__ __forceinline__ int ctl_cum(int b) { return b < 3 ? 3 * b : (b < 6 ? 9 + 12 * (b - 3) : 45); }
__device__ __forceinline__ int ctl_width(int b) { return b < 3 ? 3 : (b < 6 ? 12 : 4); }

// Prologue of one observation value (TILE: the batched kernel's layer-0 tile);
// ARITH: the prologue has per-column arithmetic (constants read from global memory).
template <bool TILE, bool ARITH>
__device__ __forceinline__ float ctl_pro(const CtlQ &q, float x, int k) {
  if constexpr (!TILE) return x;
  else if constexpr (ARITH) return prologue(q.pro, x, k);
  else return q.pro.clip ? clip_nan(x, q.pro.lo, q.pro.hi) : x;
}

// The values block BK appends to rows r < nrows (element e = r * d + c), with
// straight-line code per block and no per-element branch: one wave per SIMD has no
// other wave to cover the exec-mask round trips of a divergent if-chain (a generic
// per-element form took ~5K cycles for 16 rows at 4 waves). The thread -> element
// map is rotated by 64 * BK so that the small blocks start on different waves.
// The raw value goes to raw[r * in_dim + k] (TILE: the tile's global obs rows) and
// its prologue value to dst[r * ds + k]. NaN among the appended values of blocks
// 0-5 — where the reference's populate_buffer check exit(1)s
// (controller.hpp:57-64) — sets nanf[r] (a relaxed workgroup-scope LDS or: no fence).
// nanm: bit r set when a value of row r is NaN (OR-ed into L.nanf once per thread by
// ctl_nan_flush: a workgroup-scope LDS atomic per element, on the few addresses of 16
// rows, serialised in the LDS pipeline).
// ONE (r06): nrows * d <= nt (the batched tile: 16 rows, 256 threads), so each thread
// has at most one element of the block: straight-line predicated code instead of a loop,
// and the caller's seven blocks become one sequence the compiler can schedule as a whole
// (their LDS reads in flight together).
template <int BK, bool TILE, bool ARITH, bool ONE = false>
__device__ __forceinline__ void ctl_append_block(const CtlLds L, const CtlQ &q, bool joy, int nrows,
                                                 float *__restrict__ dst, int ds, float *__restrict__ raw, int tid,
                                                 int nt, unsigned &nanm) {
  const float *__restrict__ obs_l = L.obs;
  const float *__restrict__ st_l = L.st;
  const float *__restrict__ jy_l = L.jy;
  const float *__restrict__ act_l = L.act;
  constexpr int d = BK < 3 ? 3 : (BK < 6 ? 12 : 4);
  constexpr int cum = BK < 3 ? 3 * BK : (BK < 6 ? 9 + 12 * (BK - 3) : 45);
  const int H = q.hist, in_dim = q.in_dim;
  const int k0 = H * cum + (H - 1) * d;  // the block's first appended column
  int t = tid - (64 * BK) % nt;
  if (t < 0) t += nt;
  if constexpr (BK == 0) {  // gravity: a quad of lanes per robot (ctl_gravity_quad; nt % 4 == 0)
    for (int e = t; e < nrows * 4; e += ONE ? 1 << 30 : nt) {
      const int r = e >> 2, c = e & 3, k = k0 + c;
#if defined(GO2PI_DIAG_GRAV_TRIVIAL)  // (diagnostics: the block's cost without its arithmetic)
      const float x = st_l[r * GO2PI_CTL_STATE_DIM + c];
#else
      const float x = ctl_gravity_quad(st_l + r * GO2PI_CTL_STATE_DIM, q.g0, q.g1, q.g2, c);
#endif
      if (c < 3) {
        nanm |= (__builtin_isnan(x) ? 1u : 0u) << r;
        if constexpr (TILE) raw[r * in_dim + k] = x;
        dst[r * ds + k] = ctl_pro<TILE, ARITH>(q, x, k);
      }
    }
    return;
  }
  for (int e = t; e < nrows * d; e += ONE ? 1 << 30 : nt) {
    const int r = e / d, c = e - r * d, k = k0 + c;
    const float *st = st_l + r * GO2PI_CTL_STATE_DIM;
    float x;
    if constexpr (BK == 1) {
      x = st[4 + c];  // imu gyroscope (controller.hpp:105-109)
    } else if constexpr (BK == 2) {
      // vel_cmd from the joystick (controller.cpp:173-179); kept (the previous
      // tick's vel_cmd_) without a joystick or without axes
      x = obs_l[r * in_dim + k];
      if (joy) {
        const float *jy = jy_l + r * GO2PI_CTL_JOY_DIM;
        const float j0 = jy[0], a0 = jy[1], a1 = jy[2], a3 = jy[3];
        const double a0d = a0;
        const float sq = (float)(a0d * a0d * (a0 > 0.f ? 1.0 : -1.0) * 0.8);  // pow(axes[0], 2) * sign * 0.8
        const float cmd = c == 0 ? a1 : (c == 2 ? a3 * a1 : sq);               // axes[1], axes[3] * axes[1]
        x = j0 != 0.f ? cmd : x;
      }
    } else if constexpr (BK == 3) {
      x = (float)((double)st[7 + c] - L.q0[c]);  // q_[i] -= q0_[i] (double q0_)
    } else if constexpr (BK == 4) {
      x = st[19 + c];
    } else if constexpr (BK == 5) {
      x = act_l[r * GO2PI_CTL_DOF + c];  // action_ before act()
    } else {  // contacts: foot_force >= 22 with the FL/FR, RL/RR swap (controller.hpp:99-103)
      x = st[31 + (c ^ 1)] >= q.thr ? 1.f : 0.f;
    }
    if constexpr (BK < 6) nanm |= (__builtin_isnan(x) ? 1u : 0u) << r;
    if constexpr (TILE) raw[r * in_dim + k] = x;
    dst[r * ds + k] = ctl_pro<TILE, ARITH>(q, x, k);
  }
}

__device__ __forceinline__ void ctl_nan_flush(const CtlLds L, unsigned nanm) {
  while (nanm) {  // (a NaN observation: rare)
    const int r = __builtin_ctz(nanm);
    nanm &= nanm - 1;
    __hip_atomic_fetch_or(L.nanf + r, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
}

// The appended blocks that read no previous observation row (all but vel_cmd, block 2,
// which keeps the previous command without a joystick): they can run while the
// previous rows are still in flight (ctl_assemble_split).
template <bool TILE, bool ARITH, bool ONE = false>
__device__ __forceinline__ void ctl_append_noobs(const CtlLds L, const CtlQ &q, bool joy, int nrows,
                                                 float *__restrict__ dst, int ds, float *__restrict__ raw, int tid,
                                                 int nt, unsigned &nanm) {
  ctl_append_block<0, TILE, ARITH, ONE>(L, q, joy, nrows, dst, ds, raw, tid, nt, nanm);
  ctl_append_block<1, TILE, ARITH, ONE>(L, q, joy, nrows, dst, ds, raw, tid, nt, nanm);
  ctl_append_block<3, TILE, ARITH, ONE>(L, q, joy, nrows, dst, ds, raw, tid, nt, nanm);
  ctl_append_block<4, TILE, ARITH, ONE>(L, q, joy, nrows, dst, ds, raw, tid, nt, nanm);
  ctl_append_block<5, TILE, ARITH, ONE>(L, q, joy, nrows, dst, ds, raw, tid, nt, nanm);
  ctl_append_block<6, TILE, ARITH, ONE>(L, q, joy, nrows, dst, ds, raw, tid, nt, nanm);
}

template <bool TILE, bool ARITH>
__device__ __forceinline__ void ctl_append(const CtlLds L, const CtlQ &q, bool joy, int nrows, float *__restrict__ dst,
                                           int ds, float *__restrict__ raw, int tid, int nt) {
  unsigned nanm = 0u;
  ctl_append_noobs<TILE, ARITH>(L, q, joy, nrows, dst, ds, raw, tid, nt, nanm);
  ctl_append_block<2, TILE, ARITH>(L, q, joy, nrows, dst, ds, raw, tid, nt, nanm);
  ctl_nan_flush(L, nanm);
}

// ctl_append with one wave per block (waves 0..6 of the caller's nt = 64 * nw >= 448
// threads; tid: the caller's thread index): every branch wave-uniform, and the seven
// blocks' LDS round trips overlap across waves instead of following one another in every
// thread (the batch-1 resident kernel: ~1.5K cycles as ctl_append, seven dependent
// round trips per thread).
template <bool TILE, bool ARITH>
__device__ __forceinline__ void ctl_append_waves(const CtlLds L, const CtlQ &q, bool joy, int nrows,
                                                 float *__restrict__ dst, int ds, float *__restrict__ raw, int tid) {
  unsigned nanm = 0u;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  switch (w) {
#ifndef GO2PI_DIAG_NO_BLOCK0
    case 0: ctl_append_block<0, TILE, ARITH>(L, q, joy, nrows, dst, ds, raw, lane, 64, nanm); break;
#endif
    case 1: ctl_append_block<1, TILE, ARITH>(L, q, joy, nrows, dst, ds, raw, lane, 64, nanm); break;
    case 2: ctl_append_block<2, TILE, ARITH>(L, q, joy, nrows, dst, ds, raw, lane, 64, nanm); break;
    case 3: ctl_append_block<3, TILE, ARITH>(L, q, joy, nrows, dst, ds, raw, lane, 64, nanm); break;
    case 4: ctl_append_block<4, TILE, ARITH>(L, q, joy, nrows, dst, ds, raw, lane, 64, nanm); break;
    case 5: ctl_append_block<5, TILE, ARITH>(L, q, joy, nrows, dst, ds, raw, lane, 64, nanm); break;
    case 6: ctl_append_block<6, TILE, ARITH>(L, q, joy, nrows, dst, ds, raw, lane, 64, nanm); break;
    default: break;
  }
  ctl_nan_flush(L, nanm);
}

// The shifted values (std::shift_left by d, controller.hpp:45-52): column k of
// every row r < nrows takes the image's column k + d. The (H - 1) * 49 shifted
// columns of all rows are one flat range (row-major, so a wave's reads and the
// caller's row stores are contiguous), U elements per thread in flight: every LDS
// read issued before the first store. TILE: dst is the batched kernel's LDS tile
// — its padding columns [in_dim, in_pad) and rows [nrows, 16) are zeroed too, unless
// PAD is false (a caller whose padding stays zero and whose rows past nrows are never read).
template <bool TILE, bool ARITH, int U, bool PAD = TILE>
__device__ __forceinline__ void ctl_shift(const CtlLds L, const CtlQ &q, int nrows, float *__restrict__ dst, int ds,
                                          float *__restrict__ raw, int tid, int nt) {
  const float *__restrict__ obs_l = L.obs;
  const int H = q.hist, h1 = H - 1, in_dim = q.in_dim, nc = h1 * GO2PI_CTL_STEP_DIM, total = nrows * nc;
  const float rnc = 1.f / (float)(nc > 0 ? nc : 1);
  for (int e0 = tid; e0 < total; e0 += U * nt) {
    float x[U];
    int rr[U], kk[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int e = min(e0 + u * nt, total - 1);
      // r = e / nc exactly: (e + 0.5) / nc is >= 0.5 / nc away from an integer and
      // the float product's error is far below that here (nc <= 15 * 49, e < 16 nc)
      const int r = (int)(((float)e + 0.5f) * rnc), j = e - r * nc;
      // the j-th shifted column: block b holds (H - 1) * d of them from column H * cum
      const int b = (j >= h1 * 3) + (j >= h1 * 6) + (j >= h1 * 9) + (j >= h1 * 21) + (j >= h1 * 33) + (j >= h1 * 45);
      const int cum = ctl_cum(b), d = ctl_width(b);
      const int k = H * cum + (j - h1 * cum);
      rr[u] = r;
      kk[u] = k;
      x[u] = obs_l[r * in_dim + k + d];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (e0 + u * nt >= total) break;
      if constexpr (TILE) raw[rr[u] * in_dim + kk[u]] = x[u];
      dst[rr[u] * ds + kk[u]] = ctl_pro<TILE, ARITH>(q, x[u], kk[u]);
    }
  }
  if constexpr (TILE && PAD) {
    // sixteen threads per row, no division (r06: the two division loops this replaces
    // compiled to ~700 instructions of unrolled remainder handling): a row's padding
    // columns [in_dim, in_pad), every column of a row past nrows
    const int in_pad = q.in_pad;
    for (int i = tid; i < GO2PI_TILE_ROWS * 16; i += nt) {
      const int r = i >> 4;
      for (int c = (r < nrows ? in_dim : 0) + (i & 15); c < in_pad; c += 16) dst[r * ds + c] = 0.f;
    }
  }
}

// ctl_shift for the batched tile (r06): a thread per (shifted column, row group), its
// column's block, width and source worked out once (ctl_shift derives row, block and
// source per element), then up to four rows' reads in flight before their writes. The
// tile's padding as ctl_shift's.
template <bool ARITH>
__device__ __forceinline__ void ctl_shift_cols(const CtlLds L, const CtlQ &q, int nrows, float *__restrict__ dst,
                                               int ds, float *__restrict__ raw, int tid, int nt) {
  const float *__restrict__ obs_l = L.obs;
  const int H = q.hist, h1 = H - 1, in_dim = q.in_dim, nc = h1 * GO2PI_CTL_STEP_DIM;
  if (nc > 0) {
    const bool fit = nc <= nt;
    const int G = fit ? nt / nc : 1;  // row groups
    for (int j0 = 0; j0 < nc; j0 += fit ? nc : nt) {
      int g = 0, j = j0 + tid;
      if (fit) {
        // tid / nc exactly: (tid + 0.5) / nc is >= 0.5 / nc from an integer, far above
        // the ~1 ulp error of the hardware reciprocal at tid < 1024
        g = (int)(((float)tid + 0.5f) * __builtin_amdgcn_rcpf((float)nc));
        j = tid - g * nc;
      }
      if (g >= G || j >= nc) continue;
      const int b = (j >= h1 * 3) + (j >= h1 * 6) + (j >= h1 * 9) + (j >= h1 * 21) + (j >= h1 * 33) + (j >= h1 * 45);
      const int cum = ctl_cum(b), d = ctl_width(b);
      const int k = H * cum + (j - h1 * cum);
      const float *src = obs_l + k + d;
      int r = g;
      for (; r < nrows; r += 4 * G) {
        float x[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) x[u] = r + u * G < nrows ? src[(r + u * G) * in_dim] : 0.f;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int rr = r + u * G;
          if (rr < nrows) {
            raw[rr * in_dim + k] = x[u];
            dst[rr * ds + k] = ctl_pro<true, ARITH>(q, x[u], k);
          }
        }
      }
    }
  }
  const int in_pad = q.in_pad;
  for (int i = tid; i < GO2PI_TILE_ROWS * 16; i += nt) {
    const int r = i >> 4;
    for (int c = (r < nrows ? in_dim : 0) + (i & 15); c < in_pad; c += 16) dst[r * ds + c] = 0.f;
  }
}

// Assemble this tick's observation rows r < nrows from the LDS image (needs the
// image complete: barrier) over all nt threads of the workgroup: the appended
// values (ctl_append) and the shifted ones (ctl_shift) go to disjoint columns, so
// the two passes need no barrier between them. (The earlier form ran the seven
// history blocks one after another, each element deriving its row, block and
// source by division: ~10K cycles per 16-robot tile at 4 waves.)
// UNR: elements in flight per thread in the shift pass (fewer where registers
// are scarce: the resident kernels). A prologue with per-column arithmetic (ARITH) reads
// its constants from global memory; without one the passes touch only LDS and the
// caller's rows, so the compiler puts no vmcnt wait among them (such a wait also
// waited for the pipeline's weight fragments in flight and for the rows' stores).
template <bool TILE, int UNR = 4>
__device__ __forceinline__ void ctl_assemble_flat(const DevProgram &P, const CtlLds L, const CtlQ q, bool joy,
                                                  int nrows, float *dst, int ds, float *raw, int tid, int nt) {
    // (GO2PI_DIAG_CLOCK: thread 0's time after each pass, slots 50-51)
  if (TILE && (q.pro.sub || q.pro.div || q.pro.mul)) {
    ctl_append<TILE, true>(L, q, joy, nrows, dst, ds, raw, tid, nt);
    GO2PI_STAMP(P, tid == 0, 50);
    ctl_shift<TILE, true, UNR>(L, q, nrows, dst, ds, raw, tid, nt);
  } else {
    ctl_append<TILE, false>(L, q, joy, nrows, dst, ds, raw, tid, nt);
    GO2PI_STAMP(P, tid == 0, 50);
    ctl_shift<TILE, false, UNR>(L, q, nrows, dst, ds, raw, tid, nt);
  }
  GO2PI_STAMP(P, tid == 0, 51);
#ifdef GO2PI_DIAG_ASM2  // both passes again, warm (instruction fetch vs. work): slots 52-53
  ctl_append<TILE, false>(L, q, joy, nrows, dst, ds, raw, tid, nt);
  GO2PI_STAMP(P, tid == 0, 52);
  ctl_shift<TILE, false, UNR>(L, q, nrows, dst, ds, raw, tid, nt);
  GO2PI_STAMP(P, tid == 0, 53);
#endif
}

// ctl_assemble_flat in two parts around `mid` (the caller's wait for the previous
// observation rows and a barrier): the blocks that read only the state, joystick and
// action rows first, while the previous observation rows (the largest DMA group, issued
// last by ctl_lds_load) are still in flight; then vel_cmd and the shift pass.
template <bool TILE, class MID>
__device__ __forceinline__ void ctl_assemble_split(const DevProgram &P, const CtlLds L, const CtlQ q, bool joy,
                                                   int nrows, float *dst, int ds, float *raw, int tid, int nt,
                                                   MID &&mid) {
  unsigned nanm = 0u;
  // (the batched tile: 16 rows over 256 threads, at most one element of a block per thread)
  constexpr bool ONE = true;
  if (TILE && (q.pro.sub || q.pro.div || q.pro.mul)) {
    ctl_append_noobs<TILE, true, ONE>(L, q, joy, nrows, dst, ds, raw, tid, nt, nanm);
    mid();
    ctl_append_block<2, TILE, true, ONE>(L, q, joy, nrows, dst, ds, raw, tid, nt, nanm);
    GO2PI_STAMP(P, tid == 0, 50);
    if constexpr (TILE) ctl_shift_cols<true>(L, q, nrows, dst, ds, raw, tid, nt);
    else ctl_shift<TILE, true, 4>(L, q, nrows, dst, ds, raw, tid, nt);
  } else {
    ctl_append_noobs<TILE, false, ONE>(L, q, joy, nrows, dst, ds, raw, tid, nt, nanm);
    mid();
    ctl_append_block<2, TILE, false, ONE>(L, q, joy, nrows, dst, ds, raw, tid, nt, nanm);
    GO2PI_STAMP(P, tid == 0, 50);
    if constexpr (TILE) ctl_shift_cols<false>(L, q, nrows, dst, ds, raw, tid, nt);
    else ctl_shift<TILE, false, 4>(L, q, nrows, dst, ds, raw, tid, nt);
  }
  ctl_nan_flush(L, nanm);
  GO2PI_STAMP(P, tid == 0, 51);
}

// s_waitcnt vmcnt(n) for a run-time n (an immediate per case; n > 63 waits for 63)
__device__ __forceinline__ void vm_wait_rt(int n) {
  switch (n) {
#define GO2PI_VMW(i) \
  case i: asm volatile("s_waitcnt vmcnt(" #i ")" ::: "memory"); break;
    GO2PI_VMW(0) GO2PI_VMW(1) GO2PI_VMW(2) GO2PI_VMW(3) GO2PI_VMW(4) GO2PI_VMW(5) GO2PI_VMW(6) GO2PI_VMW(7)
    GO2PI_VMW(8) GO2PI_VMW(9) GO2PI_VMW(10) GO2PI_VMW(11) GO2PI_VMW(12) GO2PI_VMW(13) GO2PI_VMW(14) GO2PI_VMW(15)
    GO2PI_VMW(16) GO2PI_VMW(17) GO2PI_VMW(18) GO2PI_VMW(19) GO2PI_VMW(20) GO2PI_VMW(21) GO2PI_VMW(22) GO2PI_VMW(23)
    GO2PI_VMW(24) GO2PI_VMW(25) GO2PI_VMW(26) GO2PI_VMW(27) GO2PI_VMW(28) GO2PI_VMW(29) GO2PI_VMW(30) GO2PI_VMW(31)
#undef GO2PI_VMW
    default: asm volatile("s_waitcnt vmcnt(32)" ::: "memory"); break;
  }
}

// direct-to-LDS instructions glds_copy(n floats, this wave of nw) issues
__device__ __forceinline__ int glds_count(int n, int wave, int nw) {
  return n > wave * 64 ? (n - wave * 64 + nw * 64 - 1) / (nw * 64) : 0;
}

// What the final layer's store needs (controller tick), by value: the call's
// output pointers, the parameters, and this tile's LDS q0 / joystick rows.
struct CtlView {
  float *action;
  double *q_des, *kp, *kd;
  const double *q0;
  const float *jy;  // null: no joystick
  double scale, kp_run, kp_stop, kd_run;
  float lim;
  int row0;
  int on;  // 0: plain policy launch (the final layer writes `out`)
};

__device__ __forceinline__ CtlView ctl_view(const DevCtl C, const CtlLds L, int row0) {
  kparams_t &Q = *(kparams_t *)C.prm;
  return CtlView{C.action, C.q_des, C.kp, C.kd, L.q0, C.joy ? L.jy : nullptr, Q.action_scale, Q.kp_run,
                 Q.kp_stop, Q.kd_run, Q.action_limit, row0, 1};
}

// Action post-processing of robot `row`, joint n (controller.cpp:217-223, 240-248).
__device__ __forceinline__ void ctl_store(const CtlView V, int row, int n, float v) {
#pragma clang fp contract(off)  // q_des: a product then a sum, two roundings, as the reference's x86 build
  float a = v < -V.lim ? -V.lim : (V.lim < v ? V.lim : v);  // std::clamp (NaN passes through)
  const bool stop = V.jy && V.jy[(row - V.row0) * GO2PI_CTL_JOY_DIM + 4] != 0.f;
  a *= stop ? 0.f : 1.f;  // a *= joy_->buttons[0] == 0
  const size_t o = (size_t)row * GO2PI_CTL_DOF + n;
  V.action[o] = a;
  if (V.q_des) V.q_des[o] = V.q0[n] + (double)a * V.scale;
  if (V.kp) V.kp[o] = stop ? V.kp_stop : V.kp_run;
  if (V.kd) V.kd[o] = V.kd_run;
}

// The resident controller form's answer (policy_act1_kernel, CTL): each output value as
// an {epoch, 32 bits} granule at its ctl_gran offset, stored at system scope (written
// through to the host's pinned memory on its own); the host checks every tag, so no
// drain, fence or done word follows the last store. V's output pointers only say which
// outputs the call asked for. Per element the operations of ctl_store. The caller's
// consecutive threads take consecutive (row, joint) outputs: every store instruction
// then writes one contiguous range.
__device__ __forceinline__ void gran_put(unsigned long long *g, unsigned e, unsigned bits) {
  __hip_atomic_store(g, ((unsigned long long)e << 32) | bits, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
// two consecutive granules {lo, e}, {hi, e} in one 16-byte system-scope store (each
// granule checked on its own: a torn 16-byte write is harmless)
__device__ __forceinline__ void gran_put2(unsigned long long *g, unsigned e, unsigned lo, unsigned hi) {
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  const u32x4 v = {lo, e, hi, e};
  asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" ::"v"(g), "v"(v) : "memory");
}
__device__ __forceinline__ void ctl_store_gran(const CtlView V, int row, int n, float v, unsigned long long *g,
                                               const CtlGran G, unsigned e) {
#pragma clang fp contract(off)
  float a = v < -V.lim ? -V.lim : (V.lim < v ? V.lim : v);
  const bool stop = V.jy && V.jy[(row - V.row0) * GO2PI_CTL_JOY_DIM + 4] != 0.f;
  a *= stop ? 0.f : 1.f;
  const int o = row * GO2PI_CTL_DOF + n;
  gran_put(g + G.act + o, e, __float_as_uint(a));
  auto put64 = [&](int off, double x) {  // both halves' granules in one 16-byte store
    const unsigned long long b = (unsigned long long)__double_as_longlong(x);
    gran_put2(g + off + 2 * o, e, (unsigned)b, (unsigned)(b >> 32));
  };
  if (V.q_des) put64(G.qdes, V.q0[n] + (double)a * V.scale);
  if (V.kp) put64(G.kp, stop ? V.kp_stop : V.kp_run);
  if (V.kd) put64(G.kd, V.kd_run);
}

// The same for joints n .. n + 3 of one robot (n % 4 == 0, all four < 12): the
// joystick row read once, and every output as 16-byte stores (the batched kernel's
// head lane holds four consecutive joints). Per element the operations of ctl_store.
__device__ __forceinline__ void ctl_store4(const CtlView V, int row, int n, const float (&v)[4]) {
#pragma clang fp contract(off)
  const bool stop = V.jy && V.jy[(row - V.row0) * GO2PI_CTL_JOY_DIM + 4] != 0.f;
  float a[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    a[i] = v[i] < -V.lim ? -V.lim : (V.lim < v[i] ? V.lim : v[i]);
    a[i] *= stop ? 0.f : 1.f;
  }
  const size_t o = (size_t)row * GO2PI_CTL_DOF + n;
  *reinterpret_cast<float4 *>(V.action + o) = make_float4(a[0], a[1], a[2], a[3]);
  typedef double f64x2 __attribute__((ext_vector_type(2)));
  if (V.q_des) {
    f64x2 q[2];
#pragma unroll
    for (int i = 0; i < 4; ++i) q[i >> 1][i & 1] = V.q0[n + i] + (double)a[i] * V.scale;
    reinterpret_cast<f64x2 *>(V.q_des + o)[0] = q[0];
    reinterpret_cast<f64x2 *>(V.q_des + o)[1] = q[1];
  }
  if (V.kp) {
    const double k = stop ? V.kp_stop : V.kp_run;
    reinterpret_cast<f64x2 *>(V.kp + o)[0] = f64x2{k, k};
    reinterpret_cast<f64x2 *>(V.kp + o)[1] = f64x2{k, k};
  }
  if (V.kd) {
    reinterpret_cast<f64x2 *>(V.kd + o)[0] = f64x2{V.kd_run, V.kd_run};
    reinterpret_cast<f64x2 *>(V.kd + o)[1] = f64x2{V.kd_run, V.kd_run};
  }
}

}  // namespace go2pi
