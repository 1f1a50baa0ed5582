// Rotary position embedding (rotate-half form) forward / backward for gfx950, in place on strided
// Q/K views (e.g. directly inside the fused QKV GEMM output).
//
// Replaces Megatron's PyTorch-level RoPE (`--position-embedding-type rope`, `--rotary-percent`,
// /root/reference/3_training_megatron-lm/megatron/arguments.py:572-579), needed by the
// LLaMA-7B and GPT RoPE configurations.
//
// cos/sin come from a host-precomputed fp32 table [max_pos, rot/2] (Appendix B of the HIP guide:
// on-device trig turns this memory-bound op VALU-bound). Each thread rotates 8 pairs with two
// 16-byte loads (first half / second half of the rotary slice).
//
// Token t's position is (t / pos_div) % pos_mod: pos_div = 1, pos_mod = s for [b, s, ...] and
// pos_div = b for [s, b, ...] layouts.
#include "common.h"
#include "launchers.h"

namespace smdt {

template <typename T>
__global__ __launch_bounds__(256) void rope_kernel(T* __restrict__ x, int64_t ntok, int nh,
                                                   int64_t tok_stride, int64_t head_stride,
                                                   int rot, const float* __restrict__ cos_t,
                                                   const float* __restrict__ sin_t, int pos_div,
                                                   int pos_mod, float sign) {
  const int half = rot / 2;
  const int groups = half / 8;  // 8-pair groups per head
  const int64_t total = ntok * nh * groups;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * 256) {
    int gidx = (int)(i % groups);
    int64_t th = i / groups;
    int h = (int)(th % nh);
    int64_t t = th / nh;
    int pos = (int)((t / pos_div) % pos_mod);
    T* base = x + t * tok_stride + h * head_stride + gidx * 8;
    float a[8], b[8], c[8], s[8];
    load_vec<T, 8>(base, a);
    load_vec<T, 8>(base + half, b);
    load_vec<float, 8>(cos_t + (int64_t)pos * half + gidx * 8, c);
    load_vec<float, 8>(sin_t + (int64_t)pos * half + gidx * 8, s);
    float oa[8], ob[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float sn = sign * s[j];
      // [x1, x2] -> [x1 cos - x2 sin, x2 cos + x1 sin]
      oa[j] = a[j] * c[j] - b[j] * sn;
      ob[j] = b[j] * c[j] + a[j] * sn;
    }
    store_vec<T, 8>(base, oa);
    store_vec<T, 8>(base + half, ob);
  }
}

// Token-per-block form: one block per token, so the token's position (and its cos / sin rows) is
// block-uniform scalar work and the per-thread (head, group) index is 32-bit arithmetic. The
// grid-stride form above spends five 64-bit divisions / modulos per 16 elements, which made it
// VALU-bound at ~3.1 TB/s on the LLaMA-7B SFT shapes (64 q + k heads of 128,
// profiles/r4_sft_gemm_split/sft_dp8_rank_step_breakdown.txt). Measured on the NB4 SFT emulated
// DP8 rank: 20,614 / 20,617 vs 20,580 input tokens/s with the grid-stride form (same box,
// profiles/r4_rope_tok/) — the RoPE share of that step is ~1.5 %, so the gain is within noise;
// kept for its simpler index math.
template <typename T>
__global__ __launch_bounds__(256) void rope_tok_kernel(T* __restrict__ x, int nh, int64_t tok_stride,
                                                       int64_t head_stride, int rot,
                                                       const float* __restrict__ cos_t,
                                                       const float* __restrict__ sin_t, int pos_div,
                                                       int pos_mod, float sign) {
  const int half = rot / 2;
  const int groups = half / 8;
  const int64_t t = blockIdx.x;
  const int pos = (int)((t / pos_div) % pos_mod);
  const float* ct = cos_t + (int64_t)pos * half;
  const float* stb = sin_t + (int64_t)pos * half;
  T* xt = x + t * tok_stride;
  for (int i = threadIdx.x; i < nh * groups; i += 256) {
    const int h = i / groups, gidx = i - h * groups;
    T* base = xt + (int64_t)h * head_stride + gidx * 8;
    float a[8], b[8], c[8], s[8];
    load_vec<T, 8>(base, a);
    load_vec<T, 8>(base + half, b);
    load_vec<float, 8>(ct + gidx * 8, c);
    load_vec<float, 8>(stb + gidx * 8, s);
    float oa[8], ob[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float sn = sign * s[j];
      oa[j] = a[j] * c[j] - b[j] * sn;
      ob[j] = b[j] * c[j] + a[j] * sn;
    }
    store_vec<T, 8>(base, oa);
    store_vec<T, 8>(base + half, ob);
  }
}

}  // namespace smdt

using namespace smdt;

extern "C" hipError_t smdt_rope(int dtype, void* x, int64_t ntok, int nh, int64_t tok_stride,
                                int64_t head_stride, int rot, const float* cos_t,
                                const float* sin_t, int pos_div, int pos_mod, int backward,
                                hipStream_t st) {
  if (rot % 16 != 0) return hipErrorInvalidValue;
  float sign = backward ? -1.f : 1.f;
  if (ntok <= 0x7FFFFFFF && (int64_t)nh * (rot / 16) >= 64) {   // one block per token
    const dim3 g((unsigned)ntok);
    if (dtype == 1) hipLaunchKernelGGL(rope_tok_kernel<bf16>, g, dim3(256), 0, st, (bf16*)x, nh, tok_stride, head_stride, rot, cos_t, sin_t, pos_div, pos_mod, sign);
    else if (dtype == 2) hipLaunchKernelGGL(rope_tok_kernel<f16>, g, dim3(256), 0, st, (f16*)x, nh, tok_stride, head_stride, rot, cos_t, sin_t, pos_div, pos_mod, sign);
    else hipLaunchKernelGGL(rope_tok_kernel<float>, g, dim3(256), 0, st, (float*)x, nh, tok_stride, head_stride, rot, cos_t, sin_t, pos_div, pos_mod, sign);
    return hipGetLastError();
  }
  int grid = stream_grid(ntok * nh * (rot / 16), 256);
  if (dtype == 1) hipLaunchKernelGGL(rope_kernel<bf16>, dim3(grid), dim3(256), 0, st, (bf16*)x, ntok, nh, tok_stride, head_stride, rot, cos_t, sin_t, pos_div, pos_mod, sign);
  else if (dtype == 2) hipLaunchKernelGGL(rope_kernel<f16>, dim3(grid), dim3(256), 0, st, (f16*)x, ntok, nh, tok_stride, head_stride, rot, cos_t, sin_t, pos_div, pos_mod, sign);
  else hipLaunchKernelGGL(rope_kernel<float>, dim3(grid), dim3(256), 0, st, (float*)x, ntok, nh, tok_stride, head_stride, rot, cos_t, sin_t, pos_div, pos_mod, sign);
  return hipGetLastError();
}
