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

// ONNX Softplus ln(exp(x) + 1) in the overflow-free form max(x, 0) + ln(1 + exp(-|x|))
// on v_exp_f32 / v_log_f32 (~1 ulp each): the 1 + t rounding costs at most half an
// ulp of 1 (4e-8 absolute after the ln 2 scale); a NaN propagates through the log.
__device__ __forceinline__ float softplus_fast(float x) {
  const float t = __builtin_amdgcn_exp2f(-fabsf(x) * 1.4426950408889634f);
  return fmaxf(x, 0.f) + __builtin_amdgcn_logf(1.f + t) * 0.6931471805599453f;
}

// ONNX Clip (opset 11+): std::min(std::max(x, lo), hi) as onnxruntime computes it,
// so a NaN passes through (fminf / fmaxf would return the bound instead).
__device__ __forceinline__ float clip_nan(float x, float lo, float hi) {
  return x < lo ? lo : (x > hi ? hi : x);
}

// A dense layer's activation and its ONNX attributes (Elu / LeakyRelu alpha; Clip
// min / max; Selu alpha / gamma; HardSigmoid alpha / beta), Act in onnx_model.hpp.
struct ActP {
  int act;
  float alpha, beta;
};

// the kind of every activation after the six of r01-r03 (Clip, Selu, Softplus,
// HardSigmoid, HardSwish, Softsign) as one compile-time case: its epilogue applies
// act_fn per element (a branch on the uniform kind), which keeps the number of
// epilogue instantiations of every kernel template at seven
#define GO2PI_ACT_RT 100

__device__ __forceinline__ float act_fn(int act, float alpha, float beta, float x);

// Activation with the kind known at compile time: epilogues dispatch ONCE per
// tile group (a runtime switch per element made hipcc emit every activation's
// code, an IEEE divide and a vmcnt(0) wait for each of the 16 elements per lane:
// measured 4.4K cycles per layer epilogue).
template <int ACT>
__device__ __forceinline__ float act_t(const ActP &a, float x) {
#ifdef GO2PI_DIAG_NOEPI
  return x;
#endif
  const float alpha = a.alpha, beta = a.beta;
  if constexpr (ACT == 1) return x > 0.f ? x : alpha * expm1_neg(x);  // Elu (ONNX opset 6)
  else if constexpr (ACT == 2) return x > 0.f ? x : 0.f;              // Relu
  else if constexpr (ACT == 3) return tanhf(x);                       // Tanh
  else if constexpr (ACT == 4) return sigmoid_fast(x);                // Sigmoid
  else if constexpr (ACT == 5) return x >= 0.f ? x : alpha * x;       // LeakyRelu
  else if constexpr (ACT == 6) return clip_nan(x, alpha, beta);       // Clip (ReLU6: 0, 6)
  else if constexpr (ACT == 7) return x > 0.f ? beta * x : beta * (alpha * expm1_neg(x));  // Selu
  else if constexpr (ACT == 8) return softplus_fast(x);                                     // Softplus
  else if constexpr (ACT == 9) return clip_nan(alpha * x + beta, 0.f, 1.f);                // HardSigmoid
  else if constexpr (ACT == 10) return x * clip_nan(alpha * x + beta, 0.f, 1.f);           // HardSwish
  else if constexpr (ACT == 11) return x * __builtin_amdgcn_rcpf(1.f + fabsf(x));          // Softsign (rcp: ~1 ulp)
  else if constexpr (ACT == GO2PI_ACT_RT) return act_fn(a.act, alpha, beta, x);
  else return x;
}

__device__ __forceinline__ float act_fn(int act, float alpha, float beta, float x) {
  const ActP a{act, alpha, beta};
  switch (act) {
    case 1: return act_t<1>(a, x);
    case 2: return act_t<2>(a, x);
    case 3: return act_t<3>(a, x);
    case 4: return act_t<4>(a, x);
    case 5: return act_t<5>(a, x);
    case 6: return act_t<6>(a, x);
    case 7: return act_t<7>(a, x);
    case 8: return act_t<8>(a, x);
    case 9: return act_t<9>(a, x);
    case 10: return act_t<10>(a, x);
    case 11: return act_t<11>(a, x);
    default: return x;
  }
}

// Calls f(std::integral_constant<int, ACT>) for the runtime activation kind (the
// kinds past LeakyRelu share GO2PI_ACT_RT).
template <class F>
__device__ __forceinline__ void with_act(int act, F &&f) {
  switch (act) {
    case 0: f(std::integral_constant<int, 0>{}); break;
    case 1: f(std::integral_constant<int, 1>{}); break;
    case 2: f(std::integral_constant<int, 2>{}); break;
    case 3: f(std::integral_constant<int, 3>{}); break;
    case 4: f(std::integral_constant<int, 4>{}); break;
    case 5: f(std::integral_constant<int, 5>{}); break;
    default: f(std::integral_constant<int, GO2PI_ACT_RT>{}); break;
  }
}

// The action epilogue (go2pi_opts and a graph's trailing Clip / scalar Mul):
// y <- scale * clip(tanh?(y), lo, hi); the clip passes a NaN through, as ONNX Clip.
// Post: its program fields read once, by value — a loop that stores the actions
// would otherwise reload them (and wait for the scalar load) per element.
struct Post {
  int tanh;
  float lo, hi, scale;
};

__device__ __forceinline__ Post post_of(const DevProgram &P) { return Post{P.post_tanh, P.clip_lo, P.clip_hi, P.scale}; }

__device__ __forceinline__ float post_fn(const Post &q, float v) {
  if (q.tanh) v = tanhf(v);
  v = clip_nan(v, q.lo, q.hi);
  return v * q.scale;
}

__device__ __forceinline__ float post_fn(const DevProgram &P, float v) { return post_fn(post_of(P), v); }

// The prologue's program fields, read once (by value): loops that store to memory
// between elements would otherwise reload them, and a reload the compiler cannot
// prove unaliased by those stores becomes a vector load (an L2 round trip per element).
struct Pro {
  const float *sub, *div, *mul;
  int sub_b, div_b, mul_b, clip;
  float lo, hi;
};

__device__ __forceinline__ Pro pro_of(const DevProgram &P) {
  return Pro{P.pre_sub, P.pre_div, P.pre_mul, P.pre_sub_bcast, P.pre_div_bcast, P.pre_mul_bcast, P.pre_clip,
             P.obs_lo, P.obs_hi};
}

__device__ __forceinline__ float prologue(const Pro &q, float v, int k) {
  if (q.sub) v -= q.sub[q.sub_b ? 0 : k];
  if (q.div) v /= q.div[q.div_b ? 0 : k];
  if (q.mul) v *= q.mul[q.mul_b ? 0 : k];
  if (q.clip) v = clip_nan(v, q.lo, q.hi);
  return v;
}

__device__ __forceinline__ float prologue(const DevProgram &P, float v, int k) { return prologue(pro_of(P), v, k); }

// One column's prologue constants, read once for a column applied to many rows
// (the identity values where an op is absent: never applied, q's flags decide).
struct ProK {
  float sub, div, mul;
};

__device__ __forceinline__ ProK pro_k(const Pro &q, int k) {
  return ProK{q.sub ? q.sub[q.sub_b ? 0 : k] : 0.f, q.div ? q.div[q.div_b ? 0 : k] : 1.f,
              q.mul ? q.mul[q.mul_b ? 0 : k] : 1.f};
}

__device__ __forceinline__ float prologue(const Pro &q, const ProK &c, float v) {
  if (q.sub) v -= c.sub;
  if (q.div) v /= c.div;
  if (q.mul) v *= c.mul;
  if (q.clip) v = clip_nan(v, q.lo, q.hi);
  return v;
}

}  // namespace go2pi
