// HIP kernels for gfx950 (MI355X, CDNA4): the policy forward pass that the
// reference delegates to onnxruntime's CPU EP inside ONNXActor::act()
// (onnx_inference/src/cpp/onnx_actor.cpp:47 -> Gemm/Elu chain of model.onnx).
//
// 1. policy_fused_kernel<NW>  — the batched (many-robot) path.
//    One workgroup owns a tile of 16 robots for the WHOLE policy: the
//    activations of its 16 rows stay in LDS between layers (never touch HBM),
//    every layer is a strict-fp32 MFMA contraction (v_mfma_f32_16x16x4_f32:
//    A = 16 robots x 4 k from LDS, B = 4 k x 16 outputs straight from HBM/L2 in
//    the pre-packed fragment order of program.hpp), bias enters as the
//    accumulator's initial value, the activation is fused into the epilogue,
//    and the final layer writes the action rows (with the optional
//    tanh/clip/scale epilogue) directly to global memory. A recurrent policy
//    runs its GRU cell first with the hidden rows carried in LDS across ticks.
//    At batch 4096 the grid is exactly 256 workgroups = one per CU.
//
// 2. gemv_layer_kernel        — the small-batch (1..8 robots) latency path.
//    One workgroup per 16-output tile, 8 waves split the K chunks, fp32 VALU
//    dot products on the same packed fragments + wave/LDS reductions. One
//    launch per layer, captured into a hipGraph by the engine.
//
// Numerics: fp32 storage and arithmetic throughout (the f32-input MFMA is an
// exact k-ordered fmaf chain, no TF32/xf32 on gfx950). The summation order
// differs from the CPU reference, so parity is tolerance-based (north_star:
// 1e-5 fp32 vs the CPU path), while every robot row is computed with an
// identical instruction sequence wherever it sits in the batch: sharded and
// unsharded runs are bit-identical.
#include "fused_impl.hpp"

namespace go2pi {

// ---------------------------------------------------------------------------
// Small-batch GEMV layer. grid = N_pad/16 workgroups (one per 16-output tile),
// 8 waves split the K chunks. x: [B][x_stride] (device or host-mapped memory),
// y: [B][y_stride]. Layer 0 applies the prologue; the final layer the epilogue.
constexpr int GEMV_WAVES = 8;

__global__ __launch_bounds__(GEMV_WAVES * 64) void gemv_layer_kernel(DevProgram P, int layer, const float *x,
                                                                     int x_stride, float *y, int y_stride, int B) {
  extern __shared__ float4 lds4[];
  float *xs = reinterpret_cast<float *>(lds4);  // [B][K_pad]
  const DevLayer &L = P.L[layer];
  const int K_pad = L.K_pad, C = K_pad >> 4, T = L.N_pad >> 4;
  const int K = layer == 0 ? P.in_dim : P.L[layer - 1].N;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int t = blockIdx.x;
  float *part = xs + GO2PI_SMALL_MAXB * K_pad;  // [GEMV_WAVES][B][16]
  // Weights and bias do not depend on the input: issue their loads first so
  // their latency overlaps the input staging (wave w owns chunks w, w+8, ...).
  constexpr int MAXS = 8;  // chunk slots per wave: K_pad <= 8 * 8 * 16 = 1024 in registers
  const float4 *W = reinterpret_cast<const float4 *>(L.w) + (size_t)t * 64 + lane;  // chunk-major
  float4 wr[MAXS];
#pragma unroll
  for (int s = 0; s < MAXS; ++s) {
    const int c = wave + s * GEMV_WAVES;
    wr[s] = c < C ? W[(size_t)c * T * 64] : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  const float bv = (wave == 0 && lane < 16) ? L.bias[t * 16 + lane] : 0.f;
  for (int e = tid; e < B * K_pad; e += GEMV_WAVES * 64) {
    const int b = e / K_pad, k = e - b * K_pad;
    float v = 0.f;
    if (k < K) {
      v = x[(size_t)b * x_stride + k];
      if (layer == 0) v = prologue(P, v, k);
    }
    xs[b * K_pad + k] = v;
  }
  __syncthreads();
  float p[GO2PI_SMALL_MAXB];
#pragma unroll
  for (int b = 0; b < GO2PI_SMALL_MAXB; ++b) p[b] = 0.f;
  const int koff = (lane >> 4) << 2;
  auto accumulate = [&](int c, const float4 &w) {
#pragma unroll
    for (int b = 0; b < GO2PI_SMALL_MAXB; ++b) {
      if (b < B) {
        const float4 a = *reinterpret_cast<const float4 *>(xs + b * K_pad + c * 16 + koff);
        p[b] = fmaf(a.x, w.x, p[b]);
        p[b] = fmaf(a.y, w.y, p[b]);
        p[b] = fmaf(a.z, w.z, p[b]);
        p[b] = fmaf(a.w, w.w, p[b]);
      }
    }
  };
#pragma unroll
  for (int s = 0; s < MAXS; ++s) {
    const int c = wave + s * GEMV_WAVES;
    if (c < C) accumulate(c, wr[s]);
  }
  for (int c = wave + MAXS * GEMV_WAVES; c < C; c += GEMV_WAVES) accumulate(c, W[(size_t)c * T * 64]);
#pragma unroll
  for (int b = 0; b < GO2PI_SMALL_MAXB; ++b) {
    p[b] += __shfl_xor(p[b], 16);
    p[b] += __shfl_xor(p[b], 32);
  }
  if (lane < 16) {
#pragma unroll
    for (int b = 0; b < GO2PI_SMALL_MAXB; ++b)
      if (b < B) part[(wave * GO2PI_SMALL_MAXB + b) * 16 + lane] = p[b];
  }
  __syncthreads();
  if (wave == 0 && lane < 16) {
    const int n = t * 16 + lane;
    const bool last = layer == P.nl - 1;
    for (int b = 0; b < B; ++b) {
      float s = 0.f;
      for (int w2 = 0; w2 < GEMV_WAVES; ++w2) s += part[(w2 * GO2PI_SMALL_MAXB + b) * 16 + lane];
      float v = act_fn(L.act, L.alpha, L.beta, s + bv);
      if (last) {
        if (n < L.N) y[(size_t)b * y_stride + n] = post_fn(P, v);
      } else {
        y[(size_t)b * y_stride + n] = v;  // padded columns are exact zeros
      }
    }
  }
  (void)T;
}

// ---------------------------------------------------------------------------
// policy_latency_kernel — the batch-1 act() path in ONE launch (B <= 4).
// One workgroup per 16-output tile of the widest layer; each layer: the
// workgroup prefetches its weight fragments into registers, gathers the layer
// input, reduces its 16 outputs over 8 waves, and publishes them as 8-byte
// {tag, value} granules (cdna_hip_programming.md Guideline 16 recipe R2: one
// aligned agent-scope relaxed store per granule; the consumer's single wave
// re-reads until every tag equals the layer's epoch — no flag, no fence, no
// counter, correct for any workgroup->XCD placement). Tags = epoch0 + layer,
// epoch0 advanced by the host every call, so granules of earlier calls never
// match. Spins are bounded: on timeout the workgroup writes `err` and stops.
constexpr int LAT_WAVES = 8;
constexpr int LAT_MAXS = 8;  // chunk slots per wave held in registers (K_pad <= 1024)
// the wave that sums a layer's partials and publishes it: the last one, since wave 0
// alone sweeps a batch-1 layer input (its loads would complete behind its own stores)
constexpr int LAT_PW = LAT_WAVES - 1;

__device__ __forceinline__ bool sweep_layer(unsigned long long *gran, int n, unsigned tag, float *dst,
                                            unsigned *err, int lane) {
  constexpr int U = 8;  // granules per lane per batch: all loads issued before any is checked
  for (unsigned spins = 0;; ++spins) {
    bool ok = true;
    for (int base = 0; base < n; base += 64 * U) {
      unsigned long long v[U];
#pragma unroll
      for (int u = 0; u < U; ++u)  // clamped index: no branch around the loads
        v[u] = __hip_atomic_load(gran + min(base + u * 64 + lane, n - 1), __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int i = base + u * 64 + lane;
        if (i < n) {
          ok &= (unsigned)(v[u] >> 32) == tag;
          dst[i] = __uint_as_float((unsigned)v[u]);
        }
      }
    }
    if (__all(ok)) return true;
    if (spins > (1u << 22)) {  // ~seconds: a producer never ran (non-resident grid) -> give up
      if (lane == 0) __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      return false;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}

// CTL: controller tick — layer 0 assembles the observation (every workgroup,
// redundantly: 98 features), the final layer stores through ctl_store, and
// workgroup 0 (the only one of the one-tile final layer, so every other
// workgroup's reads of the previous obs / action are done by then) writes the
// new observation and status before signalling completion.
template <bool CTL>
__device__ __forceinline__ void latency_body(const DevProgram &P, const float *obs, float *act, int B,
                                             unsigned epoch0, unsigned long long *gran, int gstride, unsigned *err,
                                             unsigned *done, const DevCtl ctl) {
  extern __shared__ float4 lds4[];
  float *xs = reinterpret_cast<float *>(lds4);               // [B][K_pad] layer input
  float *part = xs + GO2PI_SMALL_MAXB * P.lds_stride;        // [waves][B][16] partial sums
  int &abort_flag = *reinterpret_cast<int *>(part + LAT_WAVES * GO2PI_SMALL_MAXB * 16);  // in the one LDS region
  // CTL only: the new raw observation rows [B][in_dim], then the LDS image of the inputs
  float *okeep = part + LAT_WAVES * GO2PI_SMALL_MAXB * 16 + 4;
  const int g = blockIdx.x, tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  if (tid == 0) abort_flag = 0;
  const CtlLds CL = ctl_lds(okeep + GO2PI_SMALL_MAXB * P.in_dim, GO2PI_SMALL_MAXB, P.in_dim);
  CtlView cv{};
  CtlQ cq{};
  if constexpr (CTL) {
    cq = ctl_q(P, ctl);
    cv = ctl_view(ctl, CL, 0);
    if (g < (P.L[0].N_pad >> 4)) {  // layer-0 WGs
      ctl_lds_load(CL, ctl, 0, B, P.in_dim, tid, wave, lane, LAT_WAVES);
      lds_dma_wait();  // (the assembly reads the image after this workgroup's next barrier)
    }
  }
  for (int l = 0; l < P.nl; ++l) {
    const DevLayer &L = P.L[l];
    const int T = L.N_pad >> 4, C = L.K_pad >> 4, K_pad = L.K_pad;
    if (g >= T) continue;  // this workgroup owns no tile of layer l
    const float4 *W = reinterpret_cast<const float4 *>(L.w) + (size_t)g * 64 + lane;
    float4 wr[LAT_MAXS];
#pragma unroll
    for (int s = 0; s < LAT_MAXS; ++s) {
      const int c = wave + s * LAT_WAVES;
      wr[s] = c < C ? W[(size_t)c * T * 64] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    const float bv = (wave == LAT_PW && lane < 16) ? L.bias[g * 16 + lane] : 0.f;
    if (l == 0) {
      const float *src = obs;
      if constexpr (CTL) {
        __syncthreads();  // the LDS image of the inputs (and the weights above) landed
        ctl_assemble_flat<false, 4>(P, CL, cq, ctl.joy != nullptr, B, okeep, P.in_dim, nullptr, tid, LAT_WAVES * 64);
        __syncthreads();
        src = okeep;
      }
      for (int e = tid; e < B * K_pad; e += LAT_WAVES * 64) {
        const int b = e / K_pad, k = e - b * K_pad;
        xs[e] = k < P.in_dim ? prologue(P, src[(size_t)b * P.in_dim + k], k) : 0.f;
      }
    } else {
      // every wave sweeps its own 512 granules (8 per lane, all in flight), not
      // wave 0 alone in B * K_pad / 512 serial rounds
      const int n = B * K_pad, lo = wave * 512;
      if (lo < n && !sweep_layer(gran + (size_t)(l - 1) * gstride + lo, min(512, n - lo), epoch0 + (unsigned)(l - 1),
                                 xs + lo, err, lane))
        abort_flag = 1;
    }
    __syncthreads();
    if (abort_flag) return;
    float p[GO2PI_SMALL_MAXB];
#pragma unroll
    for (int b = 0; b < GO2PI_SMALL_MAXB; ++b) p[b] = 0.f;
    const int koff = (lane >> 4) << 2;
#pragma unroll
    for (int s = 0; s < LAT_MAXS; ++s) {
      const int c = wave + s * LAT_WAVES;
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
#pragma unroll
    for (int b = 0; b < GO2PI_SMALL_MAXB; ++b) {
      p[b] += __shfl_xor(p[b], 16);
      p[b] += __shfl_xor(p[b], 32);
    }
    if (lane < 16) {
#pragma unroll
      for (int b = 0; b < GO2PI_SMALL_MAXB; ++b)
        if (b < B) part[(wave * GO2PI_SMALL_MAXB + b) * 16 + lane] = p[b];
    }
    lds_barrier();
    if (wave == LAT_PW && lane < 16) {
      const int n = g * 16 + lane;
      const bool last = l == P.nl - 1;
      const int la = L.act, LN = L.N;  // (read once: the stores below would make each row reload them)
      const float lal = L.alpha, lbe = L.beta;
      const Post po = post_of(P);
      for (int b = 0; b < B; ++b) {
        float s = 0.f;
        for (int w2 = 0; w2 < LAT_WAVES; ++w2) s += part[(w2 * GO2PI_SMALL_MAXB + b) * 16 + lane];
        const float v = act_fn(la, lal, lbe, s + bv);
        if (last) {
          if (n < LN) {
            if constexpr (CTL) ctl_store(cv, b, n, post_fn(po, v));
            else act[(size_t)b * LN + n] = post_fn(po, v);
          }
          if (!CTL && done && b == B - 1 && g == 0) {
            // completion word for the host's spin (instead of a stream sync): every
            // action store of this tile drained and made system-visible first
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            if (lane == 0 && T == 1) __hip_atomic_store(done, epoch0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          }
        } else {
          const unsigned long long gv = ((unsigned long long)(epoch0 + (unsigned)l) << 32) | __float_as_uint(v);
          __hip_atomic_store(gran + (size_t)l * gstride + b * L.N_pad + n, gv, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
        }
      }
    }
    lds_barrier();  // xs / part reused by the next layer (the granule stores stay in flight)
  }
  if constexpr (CTL) {
    if (g != 0) return;
    for (int e = tid; e < B * P.in_dim; e += LAT_WAVES * 64) ctl.obs[e] = okeep[e];
    if (ctl.status && tid < B) ctl.status[tid] = CL.nanf[tid];
    // completion word: every store of this workgroup drained and made system-visible first
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (done && tid == 0) __hip_atomic_store(done, epoch0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

__global__ __launch_bounds__(LAT_WAVES * 64) void policy_latency_kernel(const DevProgram *__restrict__ Pd,
                                                                        const float *obs, float *act, int B,
                                                                        unsigned epoch0, unsigned long long *gran,
                                                                        int gstride, unsigned *err, unsigned *done) {
  // the program lives in device memory (uploaded once): a ~60-byte kernarg
  // instead of the ~700-byte DevProgram keeps the per-launch host cost down
  latency_body<false>(*Pd, obs, act, B, epoch0, gran, gstride, err, done, DevCtl{});
}

__global__ __launch_bounds__(LAT_WAVES * 64) void policy_latency_ctl_kernel(const DevProgram *__restrict__ Pd, DevCtl C,
                                                                            int B, unsigned epoch0,
                                                                            unsigned long long *gran, int gstride,
                                                                            unsigned *err, unsigned *done) {
  latency_body<true>(*Pd, nullptr, nullptr, B, epoch0, gran, gstride, err, done, C);
}

int latency_grid(const DevProgram &p) {
  int grid = 1;
  for (int l = 0; l < p.nl; ++l) grid = std::max(grid, p.L[l].N_pad >> 4);
  return grid;
}

int launch_latency(const DevProgram &p, const DevProgram *p_dev, const float *obs, float *act, int batch,
                   unsigned epoch0,
                   unsigned long long *gran, int gstride, unsigned *err, unsigned *done, void *stream) {
  if (batch <= 0) return 0;
  if (batch > GO2PI_SMALL_MAXB) return (int)hipErrorInvalidValue;
  const int grid = latency_grid(p);
  const size_t lds =
      sizeof(float) * ((size_t)GO2PI_SMALL_MAXB * p.lds_stride + LAT_WAVES * GO2PI_SMALL_MAXB * 16 + 4);
  hipLaunchKernelGGL(policy_latency_kernel, dim3(grid), dim3(LAT_WAVES * 64), lds,
                     reinterpret_cast<hipStream_t>(stream), p_dev, obs, act, batch, epoch0, gran, gstride, err,
                     done);
  return (int)hipGetLastError();
}

int launch_latency_ctl(const DevProgram &p, const DevProgram *p_dev, const DevCtl &ctl, int batch, unsigned epoch0,
                       unsigned long long *gran, int gstride, unsigned *err, unsigned *done, void *stream) {
  if (batch <= 0) return 0;
  if (batch > GO2PI_SMALL_MAXB || p.L[p.nl - 1].N_pad != 16) return (int)hipErrorInvalidValue;
  const int grid = latency_grid(p);
  const size_t lds = sizeof(float) * ((size_t)GO2PI_SMALL_MAXB * p.lds_stride + LAT_WAVES * GO2PI_SMALL_MAXB * 16 + 4 +
                                      (size_t)GO2PI_SMALL_MAXB * p.in_dim + GO2PI_SMALL_MAXB +
                                      ctl_lds_floats(GO2PI_SMALL_MAXB, p.in_dim));
  hipLaunchKernelGGL(policy_latency_ctl_kernel, dim3(grid), dim3(LAT_WAVES * 64), lds,
                     reinterpret_cast<hipStream_t>(stream), p_dev, ctl, batch, epoch0, gran, gstride, err, done);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------
size_t fused_lds_bytes(const DevProgram &p, int waves) {
  // activation buffers + per-wave partial-sum scratch (head fusion: up to 2 tiles)
  // + the layer hand-off flags
  return sizeof(float) * (size_t)(2 + p.has_gru) * GO2PI_TILE_ROWS * p.lds_stride +
         sizeof(f32x4) * 64 * waves * (p.head_fuse > 1 ? p.head_fuse : 1) + sizeof(float) * GO2PI_FLAG_FLOATS +
         sizeof(float) * p.w4_bias;
}

size_t gemv_lds_bytes(const DevProgram &p, int layer) {
  return sizeof(float) * ((size_t)GO2PI_SMALL_MAXB * p.L[layer].K_pad + GEMV_WAVES * GO2PI_SMALL_MAXB * 16);
}

// The generic body's instantiations live in kernels_gen_w{4,8,16}.hip and the 4-wave
// pipeline's in kernels_w4_t{2,4,8}.hip (one translation unit each, compiled in
// parallel): gen_*<waves> / w4_*<tiles per wave>.
template <class F>
static int with_waves(int waves, F &&f) {
  switch (waves) {
    case 4: return f(std::integral_constant<int, 4>{});
    case 16: return f(std::integral_constant<int, 16>{});
    default: return f(std::integral_constant<int, 8>{});
  }
}

template <class F>
static int with_w4(const DevProgram &p, F &&f) {
  switch (p.w4_tpw) {
    case 2: return f(std::integral_constant<int, 2>{});
    case 4: return f(std::integral_constant<int, 4>{});
    default: return f(std::integral_constant<int, 8>{});
  }
}

int configure_kernels(const DevProgram &p, int waves) {
  hipError_t e = hipSuccess;
  if (waves == 4 && p.w4_tpw)
    e = (hipError_t)with_w4(p, [&](auto t) { return w4_configure<decltype(t)::value>(p); });
  else
    e = (hipError_t)with_waves(waves, [&](auto w) { return gen_configure<decltype(w)::value>(p); });
  if (e != hipSuccess) return (int)e;
  int gmax = 0;
  for (int l = 0; l < p.nl; ++l) gmax = std::max(gmax, (int)gemv_lds_bytes(p, l));
  e = hipFuncSetAttribute(reinterpret_cast<const void *>(&gemv_layer_kernel),
                          hipFuncAttributeMaxDynamicSharedMemorySize, gmax);
  return (int)e;
}

int launch_policy_fused(const DevProgram &p, const DevProgram *p_dev, int waves, const float *obs, float *act,
                        float *hidden, int batch, int steps, void *stream) {
  if (batch <= 0 || steps <= 0) return 0;
  if (waves == 4 && p.w4_tpw)
    return with_w4(p, [&](auto t) {
      return w4_launch<decltype(t)::value>(p, p_dev, obs, act, hidden, batch, steps, stream);
    });
  return with_waves(waves, [&](auto w) {
    return gen_launch<decltype(w)::value>(p, p_dev, obs, act, hidden, batch, steps, stream);
  });
}

int launch_policy_fused_ctl(const DevProgram &p, const DevProgram *p_dev, int waves, const DevCtl &ctl,
                            float *hidden, int batch, void *stream) {
  if (batch <= 0) return 0;
  const size_t lds = fused_ctl_lds_bytes(p, waves);
  if (lds > 160 * 1024) return (int)hipErrorInvalidValue;
  if (waves == 4 && p.w4_tpw)
    return with_w4(p, [&](auto t) { return w4_launch_ctl<decltype(t)::value>(p, p_dev, ctl, hidden, batch, stream); });
  return with_waves(waves, [&](auto w) {
    return gen_launch_ctl<decltype(w)::value>(p, p_dev, ctl, hidden, batch, stream);
  });
}

int launch_gemv_layer(const DevProgram &p, int layer, const float *x, int x_stride, float *y, int y_stride,
                      int batch, void *stream) {
  if (batch <= 0) return 0;
  if (batch > GO2PI_SMALL_MAXB) return (int)hipErrorInvalidValue;
  const dim3 grid(p.L[layer].N_pad >> 4);
  hipLaunchKernelGGL(gemv_layer_kernel, grid, dim3(GEMV_WAVES * 64), gemv_lds_bytes(p, layer),
                     reinterpret_cast<hipStream_t>(stream), p, layer, x, x_stride, y, y_stride, batch);
  return (int)hipGetLastError();
}

}  // namespace go2pi
