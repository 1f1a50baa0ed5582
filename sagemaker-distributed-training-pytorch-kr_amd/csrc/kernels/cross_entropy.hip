// Fused (vocab-parallel) softmax cross-entropy for gfx950.
//
// Replaces Megatron's vocab-parallel cross entropy (`parallel_output=True` at
// /root/reference/3_training_megatron-lm/pretrain_gpt.py:51-57, `--fp16-lm-cross-entropy` at
// megatron/arguments.py:992-994).
//
// Forward is ONE pass over the logits: a block of 256 threads owns a row and keeps an online
// (max, sum-exp) pair per thread over 16-byte vectors, merged across the block at the end, and
// picks up the target logit when the target falls in this rank's vocab slice. The three
// per-row statistics are what the tensor-parallel path all-reduces (MAX, then SUM, SUM).
// Backward writes (softmax - onehot) * dloss straight into the gradient buffer, which may
// alias the logits (in-place, no extra [tokens, V] allocation). Columns >= Vvalid are vocab
// padding (HF models whose vocab is padded to a multiple of 128): they count as -inf and get a
// zero gradient.
#include "common.h"
#include "launchers.h"

namespace smdt {

template <typename T>
__global__ __launch_bounds__(256) void ce_stats_kernel(const T* __restrict__ logits,
                                                       const int64_t* __restrict__ target,
                                                       int64_t rows, int V, int Vvalid,
                                                       int64_t vstart,
                                                       float* __restrict__ row_max,
                                                       float* __restrict__ row_sumexp,
                                                       float* __restrict__ row_tgt) {
  __shared__ float sm[4], ss[4];
  const int64_t row = blockIdx.x;
  if (row >= rows) return;
  const T* lr = logits + row * V;
  float m = -INFINITY, s = 0.f;
  constexpr int VE = 8;
  const int nvec = (Vvalid + VE - 1) / VE;  // vectors holding >= 1 real column (V % 8 == 0)
  for (int i = threadIdx.x; i < nvec; i += 256) {
    float v[VE];
    load_vec<T, VE, true>(lr + i * VE, v);  // logits stream once
    if ((i + 1) * VE > Vvalid) {
#pragma unroll
      for (int j = 0; j < VE; ++j)
        if (i * VE + j >= Vvalid) v[j] = -INFINITY;
    }
    float lm = v[0];
#pragma unroll
    for (int j = 1; j < VE; ++j) lm = fmaxf(lm, v[j]);
    float nm = fmaxf(m, lm);
    float acc = 0.f;
#pragma unroll
    for (int j = 0; j < VE; ++j) acc += __expf(v[j] - nm);
    s = (m == -INFINITY ? 0.f : s * __expf(m - nm)) + acc;
    m = nm;
  }
  for (int i = nvec * VE + threadIdx.x; i < Vvalid; i += 256) {
    float v = to_f32(lr[i]);
    float nm = fmaxf(m, v);
    s = (m == -INFINITY ? 0.f : s * __expf(m - nm)) + __expf(v - nm);
    m = nm;
  }
  // Merge (m, s) pairs: wave level then block level.
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    float om = __shfl_xor(m, o, 64), os = __shfl_xor(s, o, 64);
    float nm = fmaxf(m, om);
    s = (m == -INFINITY ? 0.f : s * __expf(m - nm)) + (om == -INFINITY ? 0.f : os * __expf(om - nm));
    m = nm;
  }
  if (lane == 0) {
    sm[wid] = m;
    ss[wid] = s;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float M = sm[0], S = ss[0];
    for (int w = 1; w < 4; ++w) {
      float nm = fmaxf(M, sm[w]);
      S = (M == -INFINITY ? 0.f : S * __expf(M - nm)) + (sm[w] == -INFINITY ? 0.f : ss[w] * __expf(sm[w] - nm));
      M = nm;
    }
    row_max[row] = M;
    row_sumexp[row] = S;
    int64_t t = target[row] - vstart;
    row_tgt[row] = (t >= 0 && t < Vvalid) ? to_f32(lr[t]) : 0.f;
  }
}

// dlogits[r, j] = (exp(x - gmax) / gsum - [j == target]) * dloss[r]   (rows with ignore = 0)
template <typename T>
__global__ __launch_bounds__(256) void ce_bwd_kernel(const T* __restrict__ logits,
                                                     const int64_t* __restrict__ target,
                                                     const float* __restrict__ gmax,
                                                     const float* __restrict__ gsum,
                                                     const float* __restrict__ dloss,
                                                     T* __restrict__ dlogits, int64_t rows, int V,
                                                     int Vvalid, int64_t vstart,
                                                     int64_t ignore_index) {
  const int64_t row = blockIdx.x;
  if (row >= rows) return;
  const T* lr = logits + row * V;
  T* dr = dlogits + row * V;
  const int64_t tg = target[row];
  const float g = tg == ignore_index ? 0.f : dloss[row];
  const float M = gmax[row];
  const float inv = 1.f / gsum[row];
  const int64_t t = tg - vstart;
  constexpr int VE = 8;
  const int nvec = V / VE;
  for (int i = threadIdx.x; i < nvec; i += 256) {
    float v[VE];
    load_vec<T, VE, true>(lr + i * VE, v);  // logits stream once
#pragma unroll
    for (int j = 0; j < VE; ++j) {
      float p = i * VE + j < Vvalid ? __expf(v[j] - M) * inv : 0.f;
      if (i * VE + j == t) p -= 1.f;
      v[j] = p * g;
    }
    // 6.6 GB of dlogits per step at GPT-2 345M / 64 x 1024 tokens: far past every cache level,
    // so the stores stream (nontemporal) like the loads
    if constexpr (sizeof(T) == 2) store_vec8_nt<T>(dr + i * VE, v);
    else store_vec<T, VE>(dr + i * VE, v);
  }
  for (int i = nvec * VE + threadIdx.x; i < V; i += 256) {
    float p = i < Vvalid ? __expf(to_f32(lr[i]) - M) * inv : 0.f;
    if (i == t) p -= 1.f;
    dr[i] = from_f32<T>(p * g);
  }
}

// Forward + backward in ONE pass, for a loss whose per-row dloss the caller applies elsewhere
// (ops/functional.py lm_head_cross_entropy: the row scale goes on the [tokens, hidden] side of the
// LM-head GEMM). A block of 1024 threads holds its whole row in registers (NV 16-byte vectors per
// thread, V <= NV * 8192), so the logits are read from HBM once and the row is overwritten IN PLACE
// with softmax - onehot (zero for ignored rows and padding columns); loss[row] = log(S) + M - x_t.
// Against ce_stats + ce_bwd this drops one full read of the logits (6.6 GB per GPT-2 345M step).
// amdgpu_waves_per_eu(8) caps the kernel at 64 VGPRs (62 used at NV = 7, no scratch) so TWO blocks
// share a CU and one block's reductions overlap the other's loads / stores: 3.31 -> 2.40 ms per step
// at [65536, 50304] (with 68 VGPRs only one block fit; profiles/r4_lm_head_ce/).
//
// LOCAL (the vocab-parallel form, TP > 1: parallel/tensor_parallel.VocabParallelLMHeadCE): the
// row is this rank's vocab slice [vstart, vstart + V); the kernel writes e = exp(x - m_local) in
// place (0 on padding) and the row's local statistics (m_local, sum e, the target logit if the
// target falls in this slice, else 0) to stats[0 / 1 / 2][row]. After the ranks combine their
// statistics the row scale c = exp(m_local - M) / S turns e into the softmax, and the one-hot is
// subtracted at ONE element per row — still a single pass over the logits.
template <typename T, int NV, bool LOCAL>
__global__ __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(8))) void ce_fused_kernel(T* __restrict__ logits,
                                                        const int64_t* __restrict__ target,
                                                        float* __restrict__ loss, int64_t rows,
                                                        int V, int Vvalid, int64_t ignore_index,
                                                        int64_t vstart) {
  __shared__ float red[16];
  __shared__ float xt_s;
  const int64_t row = blockIdx.x;
  if (row >= rows) return;
  T* lr = logits + row * V;
  const int64_t tg = LOCAL ? target[row] - vstart : target[row];
  const bool ign = LOCAL ? false : tg == ignore_index;
  if (threadIdx.x == 0) xt_s = (!ign && tg >= 0 && tg < Vvalid) ? to_f32(lr[tg]) : 0.f;
  const int nvec = V / 8;
  u16x8 raw[NV];
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int i = threadIdx.x + k * 1024;
    if (i < nvec) raw[k] = __builtin_nontemporal_load(reinterpret_cast<const u16x8*>(lr + i * 8));
  }
  auto val = [&](int k, int j) {
    unsigned short b = raw[k][j];
    T t;
    __builtin_memcpy(&t, &b, 2);
    return to_f32(t);
  };
  float m = -INFINITY;
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int i = threadIdx.x + k * 1024;
    if (i < nvec) {
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (i * 8 + j < Vvalid) m = fmaxf(m, val(k, j));
    }
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  m = wave_max(m);
  if (lane == 0) red[wid] = m;
  __syncthreads();
  float M = red[0];
#pragma unroll
  for (int w = 1; w < 16; ++w) M = fmaxf(M, red[w]);
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int i = threadIdx.x + k * 1024;
    if (i < nvec) {
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (i * 8 + j < Vvalid) s += __expf(val(k, j) - M);
    }
  }
  s = wave_sum(s);
  __syncthreads();  // every wave has read red[] (max) before it is reused
  if (lane == 0) red[wid] = s;
  __syncthreads();
  float S = 0.f;
#pragma unroll
  for (int w = 0; w < 16; ++w) S += red[w];
  const float inv = LOCAL ? 1.f : (ign ? 0.f : 1.f / S);
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int i = threadIdx.x + k * 1024;
    if (i < nvec) {
      float o[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int c = i * 8 + j;
        float p = c < Vvalid ? __expf(val(k, j) - M) * inv : 0.f;
        if (!LOCAL && !ign && c == tg) p -= 1.f;
        o[j] = p;
      }
      store_vec8_nt<T>(lr + i * 8, o);
    }
  }
  if (threadIdx.x == 0) {
    if constexpr (LOCAL) {   // stats = [3, rows]: local max, local sum, target logit (or 0)
      loss[row] = M;
      loss[rows + row] = S;
      loss[2 * rows + row] = xt_s;
    } else {
      loss[row] = ign ? 0.f : __logf(S) + M - xt_s;
    }
  }
}

}  // namespace smdt

using namespace smdt;

extern "C" hipError_t smdt_ce_stats(int dtype, const void* logits, const int64_t* target,
                                    int64_t rows, int V, int Vvalid, int64_t vstart,
                                    float* row_max, float* row_sumexp, float* row_tgt,
                                    hipStream_t st) {
  if (V % 8 != 0 || Vvalid < 1 || Vvalid > V) return hipErrorInvalidValue;
  if (dtype == 1) hipLaunchKernelGGL(ce_stats_kernel<bf16>, dim3(rows), dim3(256), 0, st, (const bf16*)logits, target, rows, V, Vvalid, vstart, row_max, row_sumexp, row_tgt);
  else if (dtype == 2) hipLaunchKernelGGL(ce_stats_kernel<f16>, dim3(rows), dim3(256), 0, st, (const f16*)logits, target, rows, V, Vvalid, vstart, row_max, row_sumexp, row_tgt);
  else hipLaunchKernelGGL(ce_stats_kernel<float>, dim3(rows), dim3(256), 0, st, (const float*)logits, target, rows, V, Vvalid, vstart, row_max, row_sumexp, row_tgt);
  return hipGetLastError();
}

extern "C" hipError_t smdt_ce_bwd(int dtype, const void* logits, const int64_t* target,
                                  const float* gmax, const float* gsum, const float* dloss,
                                  void* dlogits, int64_t rows, int V, int Vvalid,
                                  int64_t vstart, int64_t ignore_index, hipStream_t st) {
  if (V % 8 != 0 || Vvalid < 1 || Vvalid > V) return hipErrorInvalidValue;
  if (dtype == 1) hipLaunchKernelGGL(ce_bwd_kernel<bf16>, dim3(rows), dim3(256), 0, st, (const bf16*)logits, target, gmax, gsum, dloss, (bf16*)dlogits, rows, V, Vvalid, vstart, ignore_index);
  else if (dtype == 2) hipLaunchKernelGGL(ce_bwd_kernel<f16>, dim3(rows), dim3(256), 0, st, (const f16*)logits, target, gmax, gsum, dloss, (f16*)dlogits, rows, V, Vvalid, vstart, ignore_index);
  else hipLaunchKernelGGL(ce_bwd_kernel<float>, dim3(rows), dim3(256), 0, st, (const float*)logits, target, gmax, gsum, dloss, (float*)dlogits, rows, V, Vvalid, vstart, ignore_index);
  return hipGetLastError();
}

// local != 0: the vocab-parallel form (``loss`` = stats [3, rows], target offset by vstart)
extern "C" hipError_t smdt_ce_fused(int dtype, void* logits, const int64_t* target, float* loss,
                                    int64_t rows, int V, int Vvalid, int64_t ignore_index,
                                    int local, int64_t vstart, hipStream_t st) {
  // 16-bit logits only; V % 8 == 0 and the row must fit the registers of one block
  if (dtype != 1 && dtype != 2) return hipErrorInvalidValue;
  if (V % 8 != 0 || V > 8 * 8192 || Vvalid < 1 || Vvalid > V) return hipErrorInvalidValue;
  if (rows <= 0) return hipSuccess;
  const int nv = (V / 8 + 1023) / 1024;
#define SMDT_CE_FUSED(TT, NVV)                                                                                 \
  do {                                                                                                         \
    if (local)                                                                                                 \
      hipLaunchKernelGGL((ce_fused_kernel<TT, NVV, true>), dim3(rows), dim3(1024), 0, st, (TT*)logits, target, \
                         loss, rows, V, Vvalid, ignore_index, vstart);                                         \
    else                                                                                                       \
      hipLaunchKernelGGL((ce_fused_kernel<TT, NVV, false>), dim3(rows), dim3(1024), 0, st, (TT*)logits, target,\
                         loss, rows, V, Vvalid, ignore_index, vstart);                                         \
  } while (0)
  if (dtype == 1) {
    if (nv <= 4) SMDT_CE_FUSED(bf16, 4);
    else if (nv <= 7) SMDT_CE_FUSED(bf16, 7);
    else SMDT_CE_FUSED(bf16, 8);
  } else {
    if (nv <= 4) SMDT_CE_FUSED(f16, 4);
    else if (nv <= 7) SMDT_CE_FUSED(f16, 7);
    else SMDT_CE_FUSED(f16, 8);
  }
#undef SMDT_CE_FUSED
  return hipGetLastError();
}
