// Helpers shared by the resident kernels (resident.hip, resident_wide.hip): the
// polling wave's request sweep (a1_poll), the DPP row reductions (a1_dadd, a1_reduce)
// and the request's granule-to-LDS placement (a1_put, a1_put_ctl).
#pragma once

#include <hip/hip_runtime.h>

#include "ctl_fn.hpp"
#include "device_fn.hpp"
#include "program.hpp"

namespace go2pi {

typedef unsigned long long u64;
typedef float f32x2 __attribute__((ext_vector_type(2)));

constexpr int A1_NP = 2;  // granule loads per lane per sweep (header + <= 127 obs floats)
// threads of the form with CW compute waves (+ the polling wave)
__host__ __device__ constexpr int a1_nt(int cw) { return 64 * (1 + cw); }

// The weight register of each output: lane s of a row keeps output r(j, s) in register
// j, so that every step of the reduce-scatter adds the same register index of its
// partner (s ^ 8, then s ^ 7, s ^ 2, s ^ 1):
//   R = 8: r = j ^ 4 b3 ^ 3 b2 ^ b1,  R = 4: r = j ^ 2 b3 ^ b2,  R = 2: r = j ^ b3
// (b_i: bit i of s). After the reduce-scatter lane s holds output a1_out(0, s).
template <int R>
__device__ __forceinline__ int a1_out(int j, int s) {
  if constexpr (R == 8) return j ^ ((s >> 3) << 2) ^ (3 * ((s >> 2) & 1)) ^ ((s >> 1) & 1);
  else if constexpr (R == 4) return j ^ ((s >> 3) << 1) ^ ((s >> 2) & 1);
  else if constexpr (R == 2) return j ^ (s >> 3);
  else return 0;
}
template <int R>
__device__ __forceinline__ int a1_fin(int s) {
  return a1_out<R>(0, s);
}

// a + dpp(b) in one v_add_f32_dpp (the compiler kept each v_mov_b32_dpp apart from
// its add, and with two waves per SIMD every instruction of the chain costs issue
// slots); the s_nop covers the VALU-write -> DPP-read hazard (2 wait states)
template <int CTRL>
__device__ __forceinline__ float a1_dadd(float a, float b) {
  float r;
  if constexpr (CTRL == 0x128)
    asm volatile("s_nop 1\n\tv_add_f32_dpp %0, %1, %2 row_ror:8 row_mask:0xf bank_mask:0xf" : "=v"(r) : "v"(b), "v"(a));
  else if constexpr (CTRL == 0x141)
    asm volatile("s_nop 1\n\tv_add_f32_dpp %0, %1, %2 row_half_mirror row_mask:0xf bank_mask:0xf"
                 : "=v"(r) : "v"(b), "v"(a));
  else if constexpr (CTRL == 0x4E)
    asm volatile("s_nop 1\n\tv_add_f32_dpp %0, %1, %2 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf"
                 : "=v"(r) : "v"(b), "v"(a));
  else
    asm volatile("s_nop 1\n\tv_add_f32_dpp %0, %1, %2 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf"
                 : "=v"(r) : "v"(b), "v"(a));
  return r;
}

template <int R>
__device__ __forceinline__ float a1_reduce(float (&p)[R]) {
  if constexpr (R == 8) {
#pragma unroll
    for (int j = 0; j < 4; ++j) p[j] = a1_dadd<0x128>(p[j], p[j + 4]);  // row_ror:8 (lane s ^ 8)
    p[0] = a1_dadd<0x141>(p[0], p[2]);                                  // row_half_mirror (s ^ 7 within 8)
    p[1] = a1_dadd<0x141>(p[1], p[3]);
    p[0] = a1_dadd<0x4E>(p[0], p[1]);  // quad_perm [2, 3, 0, 1] (s ^ 2)
  } else if constexpr (R == 4) {
    p[0] = a1_dadd<0x128>(p[0], p[2]);
    p[1] = a1_dadd<0x128>(p[1], p[3]);
    p[0] = a1_dadd<0x141>(p[0], p[1]);
    p[0] = a1_dadd<0x4E>(p[0], p[0]);
  } else if constexpr (R == 2) {
    p[0] = a1_dadd<0x128>(p[0], p[1]);
    p[0] = a1_dadd<0x141>(p[0], p[0]);
    p[0] = a1_dadd<0x4E>(p[0], p[0]);
  } else {
    p[0] = a1_dadd<0x128>(p[0], p[0]);
    p[0] = a1_dadd<0x141>(p[0], p[0]);
    p[0] = a1_dadd<0x4E>(p[0], p[0]);
  }
  return a1_dadd<0xB1>(p[0], p[0]);  // quad_perm [1, 0, 3, 2] (s ^ 1)
}

// One sweep's granule i of the request (i = u * 64 + lane; 0 = header) into layer 0's
// input rows: flat observation index i - 1 -> row b, column k (x0 stride S).
__device__ __forceinline__ void a1_put(float *x0, int S, int in_dim, int B, int i, float v) {
  const int f = i - 1;
  const int b = B == 1 ? 0 : f / in_dim;
  x0[b * S + (f - b * in_dim)] = v;
}

// The controller form's granule i: the request's rows state [B][36] | joystick [B][5] |
// previous observation [B][in_dim] | previous action [B][12] (engine.cpp resident_serve)
// into the assembly's LDS image (ctl_fn.hpp CtlLds).
__device__ __forceinline__ void a1_put_ctl(const CtlLds &L, int in_dim, int B, int i, float v) {
  int f = i - 1;
  const int ns = B * GO2PI_CTL_STATE_DIM, nj = B * GO2PI_CTL_JOY_DIM, no = B * in_dim;
  if (f < ns) {
    L.st[f] = v;
    return;
  }
  f -= ns;
  if (f < nj) {
    L.jy[f] = v;
    return;
  }
  f -= nj;
  if (f < no) L.obs[f] = v;
  else L.act[f - no] = v;
}

// The polling wave's wait for the next request. D sweeps of the header and the
// request granules (NP loads per lane each) in flight (pinned host memory, system
// scope), each checked when it lands; the yield counter rides along with every sweep.
// 1: a request, its granules handed to put(i, value) (i = 1 .. B * per); 0: leave
// (LEAVE header, idle bound, moved yield counter, or a sweep that met a LEAVE
// granule). yield is never null (a zero word stands in): a conditional load in the
// ring made the compiler wait for every sweep in flight. v / yv: the sweep registers,
// owned by the caller and live across its whole request loop, so that after a request
// is seen the sweeps still in flight keep their registers: reused for the request word,
// the compiler made the poller wait for them (~a PCIe round trip) before the staging
// barrier. put_k(i, value, k): the same for the sweep fallback, k = the column.
template <int D, int NP, class PUT, class PUTK>
__device__ __forceinline__ int a1_poll(const u64 *q, int per, unsigned last, u64 idle_ticks, unsigned *err, int lane,
                                       unsigned &e, int &B, unsigned &word, const unsigned *yield, unsigned y0,
                                       u64 (&v)[D][NP], unsigned (&yv)[D], PUT &&put, PUTK &&put_k) {
  u64 *qm = const_cast<u64 *>(q);
  const int npoll = min(1 + per, 64 * NP);
  // the previous call's sweeps, landed long ago: used here, so their registers stay
  // theirs until now
#pragma unroll
  for (int d = 0; d < D; ++d) {
    asm volatile("" ::"v"(yv[d]));
#pragma unroll
    for (int u = 0; u < NP; ++u) asm volatile("" ::"v"(v[d][u]));
  }
  auto issue = [&](int d) {
#pragma unroll
    for (int u = 0; u < NP; ++u)
      v[d][u] = __hip_atomic_load(qm + min(u * 64 + lane, npoll - 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    yv[d] = __hip_atomic_load(const_cast<unsigned *>(yield), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  };
#pragma unroll
  for (int d = 0; d + 1 < D; ++d) issue(d);
  const u64 t0 = wall_clock64();
  for (;;) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
      issue((d + D - 1) % D);  // the newest sweep, before the oldest is looked at
      if (__builtin_amdgcn_readfirstlane(yv[d]) != y0) return 0;
      const unsigned tag = __builtin_amdgcn_readfirstlane((unsigned)(v[d][0] >> 32));
      if (tag == GO2PI_RES_LEAVE) return 0;
      if (tag != 0u && tag != last) {
        word = __builtin_amdgcn_readfirstlane((unsigned)v[d][0]);
        B = min(max((int)(word & 0xFFu), 1), GO2PI_SMALL_MAXB);
        const int n = B * per;
        if (1 + n <= npoll) {
          bool ok = true;
#pragma unroll
          for (int u = 0; u < NP; ++u) {
            const int i = u * 64 + lane;
            if (i >= 1 && i <= n) ok &= (unsigned)(v[d][u] >> 32) == tag;
          }
          if (__all(ok)) {
#pragma unroll
            for (int u = 0; u < NP; ++u) {
              const int i = u * 64 + lane;
              if (i >= 1 && i <= n) put(u, i, __uint_as_float((unsigned)v[d][u]));
            }
            e = tag;
            return 1;
          }
        } else {  // more granules than one sweep holds (B > 1 with a wide request)
          e = tag;
          for (unsigned spins = 0;; ++spins) {
            bool ok = true, lv = false;
            for (int i = 1 + lane; i <= n; i += 64) {
              const u64 g = __hip_atomic_load(qm + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
              const unsigned t = (unsigned)(g >> 32);
              ok &= t == tag;
              lv |= t == GO2PI_RES_LEAVE;
              put_k(i, __uint_as_float((unsigned)g));
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

}  // namespace go2pi
