// Bias + activation (GeLU-tanh, exact-erf GeLU, SwiGLU) forward / backward for gfx950.
//
// Replaces Megatron's TorchScript `bias_gelu` fusion (flag `--no-bias-gelu-fusion`,
// /root/reference/3_training_megatron-lm/megatron/arguments.py:819-821) and the SwiGLU
// activation used by LLaMA-style blocks (`--swiglu`, arguments.py:254-260).
//
// Layout: x is [rows, N] row-major. A block of 256 threads covers 2048 columns (one 8-element
// 16-byte chunk per thread) and a slice of rows (grid.y); a thread keeps the same columns for
// every row of its slice, so d(bias) partial sums accumulate in registers and are written once
// per block as an fp32 [grid.y, N] slab, reduced by `col_partials_reduce_kernel`.

#include "activations.h"
#include "common.h"
#include "launchers.h"

namespace smdt {

__device__ __forceinline__ float gelu_erf(float x) { return 0.5f * x * (1.f + erff(x * 0.7071067811865476f)); }
__device__ __forceinline__ float gelu_erf_grad(float x) {
  float cdf = 0.5f * (1.f + erff(x * 0.7071067811865476f));
  float pdf = 0.3989422804014327f * __expf(-0.5f * x * x);
  return cdf + x * pdf;
}
__device__ __forceinline__ float silu(float x) { return x / (1.f + __expf(-x)); }

template <int ACT>
__device__ __forceinline__ float act_fwd(float z) { return ACT == 0 ? gelu_tanh(z) : gelu_erf(z); }
template <int ACT>
__device__ __forceinline__ float act_grad(float z) { return ACT == 0 ? gelu_tanh_grad(z) : gelu_erf_grad(z); }

constexpr int kRows = 4;  // rows per thread whose loads are issued together (memory-level parallelism)

// act: 0 = gelu_tanh, 1 = gelu_erf
template <typename T, int ACT, int KR = kRows>
__global__ __launch_bounds__(256) void bias_act_fwd_kernel(const T* __restrict__ x,
                                                           const T* __restrict__ bias,
                                                           T* __restrict__ y, int64_t rows, int N,
                                                           int rows_per_slice) {
  const int ch = blockIdx.x * 256 + threadIdx.x;
  if (ch * 8 >= N) return;
  float b[8];
  if (bias) load_vec<T, 8>(bias + ch * 8, b);
  else
    for (int j = 0; j < 8; ++j) b[j] = 0.f;
  int64_t r0 = (int64_t)blockIdx.y * rows_per_slice;
  int64_t r1 = r0 + rows_per_slice < rows ? r0 + rows_per_slice : rows;
  auto row_op = [&](int64_t r, const Raw8<T>& rx) {
    float v[8];
    cvt_raw8<T>(rx, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = act_fwd<ACT>(v[j] + b[j]);
    store_vec<T, 8>(y + r * N + ch * 8, v);  // plain store: fc2's GEMM reads y right after
  };
  int64_t r = r0;
  for (; r + KR <= r1; r += KR) {
    Raw8<T> rx[KR];
#pragma unroll
    for (int u = 0; u < KR; ++u) rx[u] = load_raw8_nt(x + (r + u) * N + ch * 8);
#pragma unroll
    for (int u = 0; u < KR; ++u) row_op(r + u, rx[u]);
  }
  for (; r < r1; ++r) row_op(r, load_raw8(x + r * N + ch * 8));
}

template <typename T, int ACT, int KR = kRows>
__global__ __launch_bounds__(256) void bias_act_bwd_kernel(const T* __restrict__ dy,
                                                           const T* __restrict__ x,
                                                           const T* __restrict__ bias,
                                                           T* __restrict__ dx,
                                                           float* __restrict__ partials,
                                                           int64_t rows, int N,
                                                           int rows_per_slice) {
  const int ch = blockIdx.x * 256 + threadIdx.x;
  if (ch * 8 >= N) return;
  float b[8], acc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] = 0.f;
  if (bias) load_vec<T, 8>(bias + ch * 8, b);
  else
    for (int j = 0; j < 8; ++j) b[j] = 0.f;
  int64_t r0 = (int64_t)blockIdx.y * rows_per_slice;
  int64_t r1 = r0 + rows_per_slice < rows ? r0 + rows_per_slice : rows;
  auto row_op = [&](int64_t r, const Raw8<T>& rx, const Raw8<T>& rg) {
    float v[8], g[8];
    cvt_raw8<T>(rx, v);
    cvt_raw8<T>(rg, g);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float d = g[j] * act_grad<ACT>(v[j] + b[j]);
      v[j] = d;
      acc[j] += to_f32(from_f32<T>(d));
    }
    if constexpr (sizeof(T) == 2) store_vec8_nt<T>(dx + r * N + ch * 8, v);
    else store_vec<T, 8>(dx + r * N + ch * 8, v);
  };
  int64_t r = r0;
  for (; r + KR <= r1; r += KR) {
    Raw8<T> rx[KR], rg[KR];
#pragma unroll
    for (int u = 0; u < KR; ++u) {
      rx[u] = load_raw8_nt(x + (r + u) * N + ch * 8);
      rg[u] = load_raw8_nt(dy + (r + u) * N + ch * 8);
    }
#pragma unroll
    for (int u = 0; u < KR; ++u) row_op(r + u, rx[u], rg[u]);
  }
  for (; r < r1; ++r) row_op(r, load_raw8(x + r * N + ch * 8), load_raw8(dy + r * N + ch * 8));
  if (partials) store_vec<float, 8>(partials + (int64_t)blockIdx.y * N + ch * 8, acc);
}

// SwiGLU on a fused [rows, 2F] input laid out as [gate | up]: y = silu(gate) * up.

// SwiGLU on a [rows, 2F] input: grid.x = 8-column chunk blocks of a row, grid.y = rows (a row
// stride past 65535) — no 64-bit division / modulo per chunk as in the former grid-stride form:
// at the LLaMA-7B SFT shape (4300 x 11008) fwd 6.26 -> 6.67 TB/s, bwd 5.18 -> 5.38 TB/s
// (benchmarks/bench_elementwise.py, profiles/r4_swiglu_2d/).
template <typename T>
__global__ __launch_bounds__(256) void swiglu_fwd_kernel(const T* __restrict__ x, T* __restrict__ y,
                                                          int64_t rows, int F) {
  const int c = (blockIdx.x * 256 + threadIdx.x) * 8;
  if (c >= F) return;
  for (int64_t r = blockIdx.y; r < rows; r += gridDim.y) {
    float g[8], u[8];
    load_vec<T, 8>(x + r * 2 * F + c, g);
    load_vec<T, 8>(x + r * 2 * F + F + c, u);
#pragma unroll
    for (int j = 0; j < 8; ++j) g[j] = silu(g[j]) * u[j];
    store_vec<T, 8>(y + r * F + c, g);
  }
}

template <typename T>
__global__ __launch_bounds__(256) void swiglu_bwd_kernel(const T* __restrict__ dy, const T* __restrict__ x,
                                                          T* __restrict__ dx, int64_t rows, int F) {
  const int c = (blockIdx.x * 256 + threadIdx.x) * 8;
  if (c >= F) return;
  for (int64_t r = blockIdx.y; r < rows; r += gridDim.y) {
    float g[8], u[8], d[8], dg[8], du[8];
    load_vec<T, 8>(x + r * 2 * F + c, g);
    load_vec<T, 8>(x + r * 2 * F + F + c, u);
    load_vec<T, 8>(dy + r * F + c, d);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float sg = 1.f / (1.f + __expf(-g[j]));
      float sl = g[j] * sg;
      du[j] = d[j] * sl;
      dg[j] = d[j] * u[j] * (sg * (1.f + g[j] * (1.f - sg)));
    }
    store_vec<T, 8>(dx + r * 2 * F + c, dg);
    store_vec<T, 8>(dx + r * 2 * F + F + c, du);
  }
}



__global__ __launch_bounds__(256) void col_partials_reduce_kernel(const float* __restrict__ part,
                                                                 int nslices, int N,
                                                                 float* __restrict__ out,
                                                                 int accumulate) {
  colsum_block(part, nslices, N, N, out, accumulate != 0);
}

// Column sums of a [rows, N] matrix (a linear layer's bias gradient), phase 1: per row-slice
// fp32 partials; phase 2 is col_partials_reduce_kernel.
template <typename T>
__global__ __launch_bounds__(256) void col_sum_rows_kernel(const T* __restrict__ x,
                                                          float* __restrict__ part, int64_t rows,
                                                          int N, int rows_per_slice) {
  const int c = (blockIdx.x * 256 + threadIdx.x) * 8;
  if (c >= N) return;
  const int64_t r0 = (int64_t)blockIdx.y * rows_per_slice;
  const int64_t r1 = r0 + rows_per_slice < rows ? r0 + rows_per_slice : rows;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  auto add_row = [&](const Raw8<T>& raw) {
    float v[8];
    cvt_raw8<T>(raw, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] += v[j];
  };
  int64_t r = r0;
  for (; r + kRows <= r1; r += kRows) {  // kRows loads in flight, rows still summed in order
    Raw8<T> raw[kRows];
#pragma unroll
    for (int u = 0; u < kRows; ++u) raw[u] = load_raw8_nt(x + (r + u) * N + c);
#pragma unroll
    for (int u = 0; u < kRows; ++u) add_row(raw[u]);
  }
  for (; r < r1; ++r) add_row(load_raw8(x + r * N + c));
  float* o = part + (int64_t)blockIdx.y * N + c;
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = acc[j];
}

// Launch shapes. Launches that write d(bias) partials keep ~1024 blocks (the [slices, N] fp32
// slab is re-read by the reduce). The partial-free ones (forward, and backward when the grouped
// wgrad makes d(bias)) give every thread exactly one batch of kPF rows (all loads in flight at
// once, no loop): on [65536, 4096] bf16 fwd 5.18 -> 6.16 TB/s, bwd 5.57 -> 6.2 TB/s vs the round-4
// interim form (4x the blocks, 8-row batches), which had itself beaten the ~1024-block form by
// 2.5 % (profiles/r4_elementwise_ab/, profiles/r4_elementwise_ab/sweep2.log).
constexpr int kPF = 4;

static int pf_slices(int64_t rows, int* rows_per_slice) {
  // kPF rows per slice; more only past grid.y's 65535 slices (the kernel loops over its rows)
  int64_t rps = (rows + 65534) / 65535;
  if (rps < kPF) rps = kPF;
  *rows_per_slice = (int)rps;
  return (int)((rows + rps - 1) / rps);
}

static int act_slices(int64_t rows, int N, int* rows_per_slice) {
  int colblocks = (N / 8 + 255) / 256;
  int64_t want = (int64_t)1024 / colblocks;
  if (want < 1) want = 1;
  if (want > rows) want = rows;
  int64_t rps = (rows + want - 1) / want;
  *rows_per_slice = (int)rps;
  return (int)((rows + rps - 1) / rps);
}

}  // namespace smdt

using namespace smdt;

extern "C" int smdt_bias_act_slices(int64_t rows, int N) {
  int rps;
  return act_slices(rows, N, &rps);
}

extern "C" hipError_t smdt_bias_act_fwd(int dtype, int act, const void* x, const void* bias,
                                        void* y, int64_t rows, int N, hipStream_t st) {
  if (N % 8 != 0 || rows <= 0) return hipErrorInvalidValue;
  int rps;
  int slices = pf_slices(rows, &rps);
  dim3 grid((N / 8 + 255) / 256, slices);
#define SMDT_BA_FWD(T, A)                                                                   \
  hipLaunchKernelGGL((bias_act_fwd_kernel<T, A, kPF>), grid, dim3(256), 0, st, (const T*)x,  \
                     (const T*)bias, (T*)y, rows, N, rps)
  if (dtype == 1) { if (act == 0) SMDT_BA_FWD(bf16, 0); else SMDT_BA_FWD(bf16, 1); }
  else if (dtype == 2) { if (act == 0) SMDT_BA_FWD(f16, 0); else SMDT_BA_FWD(f16, 1); }
  else { if (act == 0) SMDT_BA_FWD(float, 0); else SMDT_BA_FWD(float, 1); }
#undef SMDT_BA_FWD
  return hipGetLastError();
}

extern "C" hipError_t smdt_bias_act_bwd(int dtype, int act, const void* dy, const void* x,
                                        const void* bias, void* dx, float* partials,
                                        float* dbias, int64_t rows, int N, int accumulate,
                                        hipStream_t st) {
  if (N % 8 != 0 || rows <= 0) return hipErrorInvalidValue;
  int rps;
  // with d(bias): the partials slab was sized by smdt_bias_act_slices (~1024 blocks)
  int slices = dbias ? act_slices(rows, N, &rps) : pf_slices(rows, &rps);
  dim3 grid((N / 8 + 255) / 256, slices);
  float* part = dbias ? partials : nullptr;
#define SMDT_BA_BWD(T, A)                                                                   \
  hipLaunchKernelGGL((bias_act_bwd_kernel<T, A, 4>), grid, dim3(256), 0, st, (const T*)dy,   \
                     (const T*)x, (const T*)bias, (T*)dx, part, rows, N, rps)
  if (dtype == 1) { if (act == 0) SMDT_BA_BWD(bf16, 0); else SMDT_BA_BWD(bf16, 1); }
  else if (dtype == 2) { if (act == 0) SMDT_BA_BWD(f16, 0); else SMDT_BA_BWD(f16, 1); }
  else { if (act == 0) SMDT_BA_BWD(float, 0); else SMDT_BA_BWD(float, 1); }
#undef SMDT_BA_BWD
  if (dbias) {
    hipLaunchKernelGGL(col_partials_reduce_kernel, dim3((N + 31) / 32), dim3(256), 0, st,
                       partials, slices, N, dbias, accumulate);
  }
  return hipGetLastError();
}

extern "C" hipError_t smdt_col_sum(const float* partials, int nslices, int N, float* out,
                                   int accumulate, hipStream_t st) {
  hipLaunchKernelGGL(col_partials_reduce_kernel, dim3((N + 31) / 32), dim3(256), 0, st,
                     partials, nslices, N, out, accumulate);
  return hipGetLastError();
}

extern "C" hipError_t smdt_bias_grad(int dtype, const void* dy, int64_t rows, int N,
                                     float* partials, float* out, int accumulate, hipStream_t st) {
  if (N % 8 != 0 || rows <= 0) return hipErrorInvalidValue;
  int rps;
  int slices = act_slices(rows, N, &rps);
  dim3 grid((N / 8 + 255) / 256, slices);
  if (dtype == 1) hipLaunchKernelGGL(col_sum_rows_kernel<bf16>, grid, dim3(256), 0, st, (const bf16*)dy, partials, rows, N, rps);
  else if (dtype == 2) hipLaunchKernelGGL(col_sum_rows_kernel<f16>, grid, dim3(256), 0, st, (const f16*)dy, partials, rows, N, rps);
  else hipLaunchKernelGGL(col_sum_rows_kernel<float>, grid, dim3(256), 0, st, (const float*)dy, partials, rows, N, rps);
  hipLaunchKernelGGL(col_partials_reduce_kernel, dim3((N + 31) / 32), dim3(256), 0, st, partials,
                     slices, N, out, accumulate);
  return hipGetLastError();
}

extern "C" hipError_t smdt_swiglu_fwd(int dtype, const void* x, void* y, int64_t rows, int F,
                                      hipStream_t st) {
  if (F % 8 != 0) return hipErrorInvalidValue;
  if (rows <= 0) return hipSuccess;
  const dim3 g2((unsigned)((F / 8 + 255) / 256), (unsigned)(rows < 65535 ? rows : 65535));
  if (dtype == 1) hipLaunchKernelGGL(swiglu_fwd_kernel<bf16>, g2, dim3(256), 0, st, (const bf16*)x, (bf16*)y, rows, F);
  else if (dtype == 2) hipLaunchKernelGGL(swiglu_fwd_kernel<f16>, g2, dim3(256), 0, st, (const f16*)x, (f16*)y, rows, F);
  else hipLaunchKernelGGL(swiglu_fwd_kernel<float>, g2, dim3(256), 0, st, (const float*)x, (float*)y, rows, F);
  return hipGetLastError();
}

extern "C" hipError_t smdt_swiglu_bwd(int dtype, const void* dy, const void* x, void* dx,
                                      int64_t rows, int F, hipStream_t st) {
  if (F % 8 != 0) return hipErrorInvalidValue;
  if (rows <= 0) return hipSuccess;
  const dim3 g2((unsigned)((F / 8 + 255) / 256), (unsigned)(rows < 65535 ? rows : 65535));
  if (dtype == 1) hipLaunchKernelGGL(swiglu_bwd_kernel<bf16>, g2, dim3(256), 0, st, (const bf16*)dy, (const bf16*)x, (bf16*)dx, rows, F);
  else if (dtype == 2) hipLaunchKernelGGL(swiglu_bwd_kernel<f16>, g2, dim3(256), 0, st, (const f16*)dy, (const f16*)x, (f16*)dx, rows, F);
  else hipLaunchKernelGGL(swiglu_bwd_kernel<float>, g2, dim3(256), 0, st, (const float*)dy, (const float*)x, (float*)dx, rows, F);
  return hipGetLastError();
}
