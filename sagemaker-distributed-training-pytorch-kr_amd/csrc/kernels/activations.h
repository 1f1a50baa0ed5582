// GeLU (tanh form) and its derivative, shared by the elementwise bias-activation kernels
// (bias_act.hip).
#pragma once
#include "common.h"

namespace smdt {

// tanh(u) = 1 - 2 / (1 + 2^(2 u log2 e)): one v_exp_f32 + one v_rcp_f32 instead of libm tanhf,
// whose ~20-instruction sequence made the bias-GeLU kernels VALU-bound at [16k, 4096]. Saturates
// to +-1 for large |u| (exp2 -> inf / 0); absolute error ~1e-7, far below bf16 resolution.
__device__ __forceinline__ float fast_tanh(float u) {
  return 1.f - 2.f * __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(u * 2.8853900817779268f));
}
__device__ __forceinline__ float gelu_tanh(float x) {
  constexpr float k0 = 0.7978845608028654f;  // sqrt(2/pi)
  constexpr float k1 = 0.044715f;
  float u = k0 * (x + k1 * x * x * x);
  return 0.5f * x * (1.f + fast_tanh(u));
}
__device__ __forceinline__ float gelu_tanh_grad(float x) {
  constexpr float k0 = 0.7978845608028654f;
  constexpr float k1 = 0.044715f;
  float x2 = x * x;
  float u = k0 * (x + k1 * x2 * x);
  float t = fast_tanh(u);
  return 0.5f * (1.f + t) + 0.5f * x * (1.f - t * t) * k0 * (1.f + 3.f * k1 * x2);
}
}  // namespace smdt
