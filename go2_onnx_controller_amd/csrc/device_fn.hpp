// Device helpers shared by kernels.hip and resident.hip: activations, the
// optional observation prologue and action epilogue (go2pi_opts).
#pragma once
#include <hip/hip_runtime.h>

#include <type_traits>

#include "program.hpp"

namespace go2pi {

// exp(x) - 1 for x <= 0 on the hardware exp2 (v_exp_f32, ~1 ulp): the literal
// ONNX Elu formula alpha * (exp(x) - 1). Absolute error <= ~1.2e-7 (one ulp of
// 1.0), far inside the 1e-5 contract, at ~4 VALU ops instead of libm's expm1f.
__device__ __forceinline__ float expm1_neg(float x) {
  return __builtin_amdgcn_exp2f(x * 1.4426950408889634f) - 1.f;
}

// sigmoid on v_exp_f32 + v_rcp_f32 (each ~1 ulp): ~2e-7 relative, no IEEE
// division sequence. exp2 of a large positive argument gives +inf -> rcp -> 0.
__device__ __forceinline__ float sigmoid_fast(float x) {
  return __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(x * -1.4426950408889634f));
}

// Activation with the kind known at compile time: epilogues dispatch ONCE per
// tile group (a runtime switch per element made hipcc emit every activation's
// code, an IEEE divide and a vmcnt(0) wait for each of the 16 elements per lane:
// measured 4.4K cycles per layer epilogue).
template <int ACT>
__device__ __forceinline__ float act_t(float alpha, float x) {
#ifdef GO2PI_DIAG_NOEPI
  return x;
#endif
  if constexpr (ACT == 1) return x > 0.f ? x : alpha * expm1_neg(x);  // Elu (ONNX opset 6)
  else if constexpr (ACT == 2) return x > 0.f ? x : 0.f;              // Relu
  else if constexpr (ACT == 3) return tanhf(x);                       // Tanh
  else if constexpr (ACT == 4) return sigmoid_fast(x);                // Sigmoid
  else if constexpr (ACT == 5) return x >= 0.f ? x : alpha * x;       // LeakyRelu
  else return x;
}

__device__ __forceinline__ float act_fn(int act, float alpha, float x) {
  switch (act) {
    case 1: return act_t<1>(alpha, x);
    case 2: return act_t<2>(alpha, x);
    case 3: return act_t<3>(alpha, x);
    case 4: return act_t<4>(alpha, x);
    case 5: return act_t<5>(alpha, x);
    default: return act_t<0>(alpha, x);
  }
}

// Calls f(std::integral_constant<int, ACT>) for the runtime activation kind.
template <class F>
__device__ __forceinline__ void with_act(int act, F &&f) {
  switch (act) {
    case 1: f(std::integral_constant<int, 1>{}); break;
    case 2: f(std::integral_constant<int, 2>{}); break;
    case 3: f(std::integral_constant<int, 3>{}); break;
    case 4: f(std::integral_constant<int, 4>{}); break;
    case 5: f(std::integral_constant<int, 5>{}); break;
    default: f(std::integral_constant<int, 0>{}); break;
  }
}

__device__ __forceinline__ float post_fn(const DevProgram &P, float v) {
  if (P.post_tanh) v = tanhf(v);
  v = fminf(fmaxf(v, P.clip_lo), P.clip_hi);
  return v * P.scale;
}

__device__ __forceinline__ float prologue(const DevProgram &P, float v, int k) {
  if (P.pre_sub) v -= P.pre_sub[P.pre_sub_bcast ? 0 : k];
  if (P.pre_div) v /= P.pre_div[P.pre_div_bcast ? 0 : k];
  if (P.obs_clip > 0.f) v = fminf(fmaxf(v, -P.obs_clip), P.obs_clip);
  return v;
}

}  // namespace go2pi
