// Scaled (masked / causal) softmax forward + backward for gfx950.
//
// The MI355X-native replacement for Megatron's `scaled_upper_triang_masked_softmax`,
// `scaled_masked_softmax` and `scaled_softmax` CUDA extensions (enabled by
// `masked_softmax_fusion`, /root/reference/3_training_megatron-lm/megatron/arguments.py:814-818).
//
// One wave64 owns one row of length sk (sk <= 4096): each lane holds C chunks of 8 elements in
// registers (16-byte loads), max and sum reduce across the 64 lanes, and the row is read and
// written exactly once. In causal mode row i only needs columns 0..i: chunks entirely above
// the diagonal are neither loaded nor exponentiated (they are written as zeros), which skips
// ~half of the loads and transcendental work for square causal inputs.
//
// mode 0: no mask; mode 1: causal (upper triangle masked, Megatron semantic: key j > query i);
// mode 2: explicit uint8 mask [mb, 1, sq, sk] broadcast over heads (1 = masked).
#include "common.h"
#include "launchers.h"

namespace smdt {

template <typename T, int C, int MODE>
__global__ __launch_bounds__(256) void softmax_fwd_kernel(const T* __restrict__ x,
                                                          const uint8_t* __restrict__ mask,
                                                          T* __restrict__ y, int64_t rows, int sq,
                                                          int sk, int heads, float scale) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int qi = (int)(row % sq);
  const int nchunk = sk / 8;
  const T* xr = x + row * sk;
  T* yr = y + row * sk;
  const uint8_t* mr = nullptr;
  if (MODE == 2) {
    int64_t bh = row / sq;
    int64_t b = bh / heads;
    mr = mask + (b * sq + qi) * (int64_t)sk;
  }
  // Number of valid columns for causal rows.
  const int valid = MODE == 1 ? (qi + 1 < sk ? qi + 1 : sk) : sk;
  float v[C][8];
  float mx = -INFINITY;
#pragma unroll
  for (int c = 0; c < C; ++c) {
    const int ch = c * 64 + lane;
    const int col0 = ch * 8;
    if (ch < nchunk && col0 < valid) {
      load_vec<T, 8>(xr + col0, v[c]);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        bool m = false;
        if (MODE == 1) m = col0 + j >= valid;
        if (MODE == 2) m = mr[col0 + j] != 0;
        v[c][j] = m ? -INFINITY : v[c][j] * scale;
        mx = fmaxf(mx, v[c][j]);
      }
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[c][j] = -INFINITY;
    }
  }
  mx = wave_max(mx);
  float sum = 0.f;
  // A fully-masked row (possible with explicit masks) produces zeros, matching Megatron.
  const bool all_masked = mx == -INFINITY;
#pragma unroll
  for (int c = 0; c < C; ++c) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float e = (all_masked || v[c][j] == -INFINITY) ? 0.f : __expf(v[c][j] - mx);
      v[c][j] = e;
      sum += e;
    }
  }
  sum = wave_sum(sum);
  const float inv = sum > 0.f ? 1.f / sum : 0.f;
#pragma unroll
  for (int c = 0; c < C; ++c) {
    const int ch = c * 64 + lane;
    if (ch < nchunk) {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[c][j] *= inv;
      store_vec<T, 8>(yr + ch * 8, v[c]);
    }
  }
}

// dx = scale * y * (dy - sum(dy * y)); causal rows skip the all-zero upper chunks.
template <typename T, int C, int MODE>
__global__ __launch_bounds__(256) void softmax_bwd_kernel(const T* __restrict__ dy,
                                                          const T* __restrict__ y,
                                                          T* __restrict__ dx, int64_t rows,
                                                          int sq, int sk, float scale) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int qi = (int)(row % sq);
  const int nchunk = sk / 8;
  const int valid = MODE == 1 ? (qi + 1 < sk ? qi + 1 : sk) : sk;
  float yv[C][8], gv[C][8];
  float dot = 0.f;
#pragma unroll
  for (int c = 0; c < C; ++c) {
    const int ch = c * 64 + lane;
    if (ch < nchunk && ch * 8 < valid) {
      load_vec<T, 8>(y + row * sk + ch * 8, yv[c]);
      load_vec<T, 8>(dy + row * sk + ch * 8, gv[c]);
#pragma unroll
      for (int j = 0; j < 8; ++j) dot += yv[c][j] * gv[c][j];
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) yv[c][j] = gv[c][j] = 0.f;
    }
  }
  dot = wave_sum(dot);
#pragma unroll
  for (int c = 0; c < C; ++c) {
    const int ch = c * 64 + lane;
    if (ch < nchunk) {
      float o[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = scale * yv[c][j] * (gv[c][j] - dot);
      store_vec<T, 8>(dx + row * sk + ch * 8, o);
    }
  }
}

template <typename T, int MODE>
static hipError_t softmax_fwd_c(int C, dim3 grid, hipStream_t st, const T* x, const uint8_t* m,
                                T* y, int64_t rows, int sq, int sk, int heads, float scale) {
#define SMDT_SM_FWD(CC)                                                                   \
  case CC:                                                                                \
    hipLaunchKernelGGL((softmax_fwd_kernel<T, CC, MODE>), grid, dim3(256), 0, st, x, m, y, \
                       rows, sq, sk, heads, scale);                                       \
    break;
  switch (C) {
    SMDT_SM_FWD(1) SMDT_SM_FWD(2) SMDT_SM_FWD(4) SMDT_SM_FWD(8)
    default: return hipErrorInvalidValue;
  }
#undef SMDT_SM_FWD
  return hipGetLastError();
}

template <typename T, int MODE>
static hipError_t softmax_bwd_c(int C, dim3 grid, hipStream_t st, const T* dy, const T* y, T* dx,
                                int64_t rows, int sq, int sk, float scale) {
#define SMDT_SM_BWD(CC)                                                                    \
  case CC:                                                                                 \
    hipLaunchKernelGGL((softmax_bwd_kernel<T, CC, MODE>), grid, dim3(256), 0, st, dy, y, dx, \
                       rows, sq, sk, scale);                                               \
    break;
  switch (C) {
    SMDT_SM_BWD(1) SMDT_SM_BWD(2) SMDT_SM_BWD(4) SMDT_SM_BWD(8)
    default: return hipErrorInvalidValue;
  }
#undef SMDT_SM_BWD
  return hipGetLastError();
}

static int softmax_chunks(int sk) {
  int c = (sk / 8 + 63) / 64;
  int p = 1;
  while (p < c) p <<= 1;
  return p;
}

template <typename T>
static hipError_t softmax_fwd_t(int mode, const void* x, const uint8_t* m, void* y, int64_t rows,
                                int sq, int sk, int heads, float scale, hipStream_t st) {
  int C = softmax_chunks(sk);
  dim3 grid((unsigned)((rows + 3) / 4));
  if (mode == 0) return softmax_fwd_c<T, 0>(C, grid, st, (const T*)x, m, (T*)y, rows, sq, sk, heads, scale);
  if (mode == 1) return softmax_fwd_c<T, 1>(C, grid, st, (const T*)x, m, (T*)y, rows, sq, sk, heads, scale);
  return softmax_fwd_c<T, 2>(C, grid, st, (const T*)x, m, (T*)y, rows, sq, sk, heads, scale);
}

template <typename T>
static hipError_t softmax_bwd_t(int mode, const void* dy, const void* y, void* dx, int64_t rows,
                                int sq, int sk, float scale, hipStream_t st) {
  int C = softmax_chunks(sk);
  dim3 grid((unsigned)((rows + 3) / 4));
  if (mode == 1) return softmax_bwd_c<T, 1>(C, grid, st, (const T*)dy, (const T*)y, (T*)dx, rows, sq, sk, scale);
  return softmax_bwd_c<T, 0>(C, grid, st, (const T*)dy, (const T*)y, (T*)dx, rows, sq, sk, scale);
}

}  // namespace smdt

using namespace smdt;

extern "C" hipError_t smdt_softmax_fwd(int dtype, int mode, const void* x, const uint8_t* mask,
                                       void* y, int64_t rows, int sq, int sk, int heads,
                                       float scale, hipStream_t st) {
  if (sk % 8 != 0 || sk > 4096) return hipErrorInvalidValue;
  if (dtype == 1) return softmax_fwd_t<bf16>(mode, x, mask, y, rows, sq, sk, heads, scale, st);
  if (dtype == 2) return softmax_fwd_t<f16>(mode, x, mask, y, rows, sq, sk, heads, scale, st);
  return softmax_fwd_t<float>(mode, x, mask, y, rows, sq, sk, heads, scale, st);
}

extern "C" hipError_t smdt_softmax_bwd(int dtype, int mode, const void* dy, const void* y,
                                       void* dx, int64_t rows, int sq, int sk, float scale,
                                       hipStream_t st) {
  if (sk % 8 != 0 || sk > 4096) return hipErrorInvalidValue;
  // The explicit-mask backward is mask-free: masked probabilities are exactly zero.
  if (dtype == 1) return softmax_bwd_t<bf16>(mode, dy, y, dx, rows, sq, sk, scale, st);
  if (dtype == 2) return softmax_bwd_t<f16>(mode, dy, y, dx, rows, sq, sk, scale, st);
  return softmax_bwd_t<float>(mode, dy, y, dx, rows, sq, sk, scale, st);
}
