// Fused (residual + bias + dropout) -> LayerNorm / RMSNorm, forward and backward, for gfx950.
//
// Replaces apex `fused_layer_norm_cuda` and Megatron's bias-dropout-add + LayerNorm pair
// (flags `--no-persist-layer-norm`, `--no-bias-dropout-fusion`,
// /root/reference/3_training_megatron-lm/megatron/arguments.py:822-824, :843-847).
//
// Design (CDNA4-first, not a warp-per-row translation):
//  * A row is owned by a group of G threads: G = 64 (one wave64) for H <= 2048, G = 256
//    (a whole 4-wave block, LDS reduction) above that. Each thread keeps C chunks of 8
//    contiguous elements in registers (16-byte global_load_dwordx4 per chunk for 16-bit
//    types), so the row is read from HBM exactly once.
//  * With a fixed row->lane mapping, a lane owns the same columns for every row it sees,
//    so dgamma / dbeta / dbias partial sums stay in registers across all rows handled by
//    the wave and are flushed once per block -> [nblocks, H] fp32 partials, summed by a
//    second tiny kernel (no float atomics; bitwise reproducible).
//  * Dropout uses a stateless keyed hash of (row, col) (see dropout_mask8), so the backward
//    pass recomputes the mask instead of storing it.
#include "common.h"
#include "launchers.h"

namespace smdt {

struct LnFwdArgs {
  const void* x;      // [rows, H]  input (pre-residual branch output)
  const void* res;    // [rows, H]  residual (optional)
  const void* bias;   // [H]        bias added to x before dropout (optional)
  const void* gamma;  // [H]
  const void* beta;   // [H] (optional; ignored for RMSNorm)
  void* y;            // [rows, H]  normalised output
  void* s_out;        // [rows, H]  residual + dropout(x + bias) (when res/bias/dropout present)
  float* mean;        // [rows] (LayerNorm only)
  float* rstd;        // [rows]
  int64_t rows;
  int H;
  float eps;
  float p_drop;
  uint64_t seed, offset;
  int rms;
  const uint32_t* step;  // graph-safe RNG step counter (smdt_set_rng_step), may be null
  const void* x2;        // [rows, H] optional second summand of x (a reduce-scatter's incoming
                         // partial: x + x2 is the row-parallel output, added here instead of in
                         // a separate pass)
};

struct LnBwdArgs {
  const void* dy;     // [rows, H] grad of normalised output
  const void* ds_in;  // [rows, H] extra grad flowing into s from the residual stream (optional)
  const void* s;      // [rows, H] the LayerNorm input saved by forward
  const void* gamma;
  const float* mean;
  const float* rstd;
  void* ds_out;       // [rows, H] grad wrt LN input (+ ds_in) == grad wrt residual
  void* dx_out;       // [rows, H] grad wrt x (dropout-masked ds); may alias ds_out when p == 0
  float* partials;    // [nblocks, 3, H] fp32 (dgamma, dbeta, dbias)
  int64_t rows;
  int H;
  float p_drop;
  uint64_t seed, offset;
  int rms;
  int want_dbias;
  int nblocks;
  const uint32_t* step;
  const void* dy2;    // [rows, H] optional second summand of dy (a backward reduce-scatter's
                      // incoming partial, added here instead of in a separate pass)
};

template <int G>
__device__ __forceinline__ float group_sum(float v, float* scratch) {
  if constexpr (G == 64) {
    return wave_sum(v);
  } else {
    return block_sum(v, scratch, G / 64);
  }
}

// Hidden-dropout keep mask: one murmur3-finalizer hash per element PAIR (counter = linear pair
// index, keyed by (seed, offset)) and a 16-bit threshold per element; the realised drop rate
// thr / 65536 is what the keep scale uses. About 6x less VALU per element than Philox-4x32-7,
// which left the fused LN kernels VALU-bound; forward and backward re-derive the same mask.
__device__ __forceinline__ uint32_t fmix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x85EBCA6Bu;
  x ^= x >> 13;
  x *= 0xC2B2AE35u;
  return x ^ (x >> 16);
}
__device__ __forceinline__ uint32_t drop_thr16(float p) { return (uint32_t)(p * 65536.f + 0.5f); }
__device__ __forceinline__ float drop_scale16(uint32_t thr) { return 65536.f / (65536.f - (float)thr); }
__device__ __forceinline__ uint32_t ln_drop_key(uint64_t seed, uint64_t offset, const uint32_t* step) {
  const uint32_t k = fmix32((uint32_t)seed ^ fmix32((uint32_t)(seed >> 32) + 0x9E3779B9u * ((uint32_t)offset + 1u)) ^
                            fmix32((uint32_t)(offset >> 32) + 0x27D4EB2Fu));
  return step ? k ^ fmix32(*step * 0x9E3779B1u + 0x85EBCA77u) : k;
}
// keep[j] (1 / 0) for the 8 elements starting at (row, col), col % 8 == 0.
__device__ __forceinline__ void dropout_mask8(uint32_t key, int64_t row, int H, int col, uint32_t thr,
                                              float (&keep)[8]) {
  const uint64_t pair = ((uint64_t)row * (uint64_t)H + (uint64_t)col) >> 1;
  const uint32_t k = key ^ ((uint32_t)(pair >> 32) * 0x9E3779B1u);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const uint32_t h = fmix32(((uint32_t)pair + (uint32_t)j) ^ k);
    keep[2 * j] = (h & 0xFFFFu) >= thr ? 1.f : 0.f;
    keep[2 * j + 1] = (h >> 16) >= thr ? 1.f : 0.f;
  }
}

template <typename T, typename W, int G, int C>
__global__ __launch_bounds__(256) void ln_fwd_kernel(LnFwdArgs a) {
  __shared__ float scratch[8];
  const int H = a.H;
  const int tid_in_group = threadIdx.x % G;
  const int groups_per_block = 256 / G;
  const int group = threadIdx.x / G;
  const int nchunk = H / 8;
  const bool has_res = a.res != nullptr;
  const bool has_bias = a.bias != nullptr;
  const bool drop = a.p_drop > 0.f;
  const bool write_s = a.s_out != nullptr;
  const uint32_t dthr = drop ? drop_thr16(a.p_drop) : 0u;
  const uint32_t dkey = drop ? ln_drop_key(a.seed, a.offset, a.step) : 0u;
  const float keep_scale = drop ? drop_scale16(dthr) : 1.f;

  // gamma / beta / bias are row-invariant: load once.
  float g[C][8], b[C][8], bi[C][8];
#pragma unroll
  for (int c = 0; c < C; ++c) {
    int ch = c * G + tid_in_group;
    if (ch < nchunk) {
      load_vec<W, 8>((const W*)a.gamma + ch * 8, g[c]);
      if (!a.rms && a.beta) load_vec<W, 8>((const W*)a.beta + ch * 8, b[c]);
      else
        for (int j = 0; j < 8; ++j) b[c][j] = 0.f;
      if (has_bias) load_vec<W, 8>((const W*)a.bias + ch * 8, bi[c]);
      else
        for (int j = 0; j < 8; ++j) bi[c][j] = 0.f;
    }
  }

  for (int64_t row = (int64_t)blockIdx.x * groups_per_block + group; row < a.rows;
       row += (int64_t)gridDim.x * groups_per_block) {
    const T* xr = (const T*)a.x + row * H;
    float v[C][8];
    float sum = 0.f;
#pragma unroll
    for (int c = 0; c < C; ++c) {
      int ch = c * G + tid_in_group;
      if (ch < nchunk) {
        load_vec<T, 8, true>(xr + ch * 8, v[c]);  // streamed once: nontemporal
        if (a.x2 != nullptr) {
          float u[8];
          load_vec<T, 8, true>((const T*)a.x2 + row * H + ch * 8, u);
          for (int j = 0; j < 8; ++j) v[c][j] += u[j];
        }
        if (has_bias)
          for (int j = 0; j < 8; ++j) v[c][j] += bi[c][j];
        if (drop) {
          float keep[8];
          dropout_mask8(dkey, row, H, ch * 8, dthr, keep);
          for (int j = 0; j < 8; ++j) v[c][j] *= keep[j] * keep_scale;
        }
        if (has_res) {
          float r[8];
          load_vec<T, 8, true>((const T*)a.res + row * H + ch * 8, r);
          for (int j = 0; j < 8; ++j) v[c][j] += r[j];
        }
        if (write_s) {
          // Round the residual stream to T before normalising so forward and the
          // saved tensor used by backward agree exactly.
          store_vec<T, 8>((T*)a.s_out + row * H + ch * 8, v[c]);
#pragma unroll
          for (int j = 0; j < 8; ++j) v[c][j] = to_f32(from_f32<T>(v[c][j]));
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) sum += v[c][j];
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[c][j] = 0.f;
      }
    }
    float mu = 0.f;
    if (!a.rms) {
      mu = group_sum<G>(sum, scratch) / (float)H;
    }
    float sq = 0.f;
#pragma unroll
    for (int c = 0; c < C; ++c) {
      int ch = c * G + tid_in_group;
      if (ch < nchunk) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          float d = v[c][j] - mu;
          sq += d * d;
        }
      }
    }
    float var = group_sum<G>(sq, scratch) / (float)H;
    float rs = rsqrtf(var + a.eps);
    if (tid_in_group == 0) {
      if (!a.rms) a.mean[row] = mu;
      a.rstd[row] = rs;
    }
    T* yr = (T*)a.y + row * H;
#pragma unroll
    for (int c = 0; c < C; ++c) {
      int ch = c * G + tid_in_group;
      if (ch < nchunk) {
        float o[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = (v[c][j] - mu) * rs * g[c][j] + b[c][j];
        store_vec<T, 8>(yr + ch * 8, o);
      }
    }
  }
}

template <typename T, typename W, int G, int C>
__global__ __launch_bounds__(256) void ln_bwd_kernel(LnBwdArgs a) {
  __shared__ float scratch[8];
  __shared__ float colbuf[3][8 * 256];  // per-group partial columns for the block flush
  const int H = a.H;
  const int tid_in_group = threadIdx.x % G;
  const int groups_per_block = 256 / G;
  const int group = threadIdx.x / G;
  const int nchunk = H / 8;
  const bool drop = a.p_drop > 0.f;
  const uint32_t dthr = drop ? drop_thr16(a.p_drop) : 0u;
  const uint32_t dkey = drop ? ln_drop_key(a.seed, a.offset, a.step) : 0u;
  const float keep_scale = drop ? drop_scale16(dthr) : 1.f;
  const bool has_dsin = a.ds_in != nullptr;
  const bool separate_dx = a.dx_out != nullptr && a.dx_out != a.ds_out;

  float g[C][8];
  float pg[C][8], pb[C][8], pbi[C][8];
#pragma unroll
  for (int c = 0; c < C; ++c) {
    int ch = c * G + tid_in_group;
#pragma unroll
    for (int j = 0; j < 8; ++j) pg[c][j] = pb[c][j] = pbi[c][j] = 0.f;
    if (ch < nchunk) load_vec<W, 8>((const W*)a.gamma + ch * 8, g[c]);
  }

  // Software pipeline over the group's rows: the NEXT row's s / dy / ds_in (raw 16-byte vectors)
  // and its mean / rstd are loaded before the current row's two cross-lane reductions, so every
  // lane keeps two rows of loads in flight (one row in flight left this kernel at ~3 TB/s).
  const T* __restrict__ sp = (const T*)a.s;
  const T* __restrict__ dyp = (const T*)a.dy;
  const T* __restrict__ dip = (const T*)a.ds_in;
  const T* __restrict__ dy2p = (const T*)a.dy2;
  const bool has_dy2 = dy2p != nullptr;
  const int64_t rstep = (int64_t)gridDim.x * groups_per_block;
  Raw8<T> ns[C], ndy[C], ndi[C], ndy2[C];
#pragma unroll
  for (int c = 0; c < C; ++c) ns[c] = ndy[c] = ndi[c] = ndy2[c] = Raw8<T>{};
  float nmu = 0.f, nrs = 0.f;
  auto fetch = [&](int64_t r) {
#pragma unroll
    for (int c = 0; c < C; ++c) {
      const int ch = c * G + tid_in_group;
      if (ch < nchunk) {
        ns[c] = load_raw8_nt(sp + r * H + ch * 8);  // streamed once: nontemporal
        ndy[c] = load_raw8_nt(dyp + r * H + ch * 8);
        if (has_dsin) ndi[c] = load_raw8_nt(dip + r * H + ch * 8);
        if (has_dy2) ndy2[c] = load_raw8_nt(dy2p + r * H + ch * 8);
      }
    }
    nmu = a.rms ? 0.f : a.mean[r];
    nrs = a.rstd[r];
  };
  int64_t row = (int64_t)blockIdx.x * groups_per_block + group;
  if (row < a.rows) fetch(row);
  for (; row < a.rows; row += rstep) {
    Raw8<T> cs[C], cdy[C], cdi[C], cdy2[C];
#pragma unroll
    for (int c = 0; c < C; ++c) {
      cs[c] = ns[c];
      cdy[c] = ndy[c];
      cdi[c] = ndi[c];
      cdy2[c] = ndy2[c];
    }
    const float mu = nmu;
    const float rs = nrs;
    if (row + rstep < a.rows) fetch(row + rstep);
    float xh[C][8], dyg[C][8];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int c = 0; c < C; ++c) {
      int ch = c * G + tid_in_group;
      if (ch < nchunk) {
        float dy[8];
        cvt_raw8<T>(cs[c], xh[c]);
        cvt_raw8<T>(cdy[c], dy);
        if (has_dy2) {
          float d2[8];
          cvt_raw8<T>(cdy2[c], d2);
#pragma unroll
          for (int j = 0; j < 8; ++j) dy[j] += d2[j];
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          xh[c][j] = (xh[c][j] - mu) * rs;
          dyg[c][j] = dy[j] * g[c][j];
          pg[c][j] += dy[j] * xh[c][j];
          pb[c][j] += dy[j];
          s1 += dyg[c][j];
          s2 += dyg[c][j] * xh[c][j];
        }
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) xh[c][j] = dyg[c][j] = 0.f;
      }
    }
    const float m1 = a.rms ? 0.f : group_sum<G>(s1, scratch) / (float)H;
    const float m2 = group_sum<G>(s2, scratch) / (float)H;
#pragma unroll
    for (int c = 0; c < C; ++c) {
      int ch = c * G + tid_in_group;
      if (ch < nchunk) {
        float ds[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) ds[j] = rs * (dyg[c][j] - m1 - xh[c][j] * m2);
        if (has_dsin) {
          float e[8];
          cvt_raw8<T>(cdi[c], e);
#pragma unroll
          for (int j = 0; j < 8; ++j) ds[j] += e[j];
        }
        store_vec<T, 8>((T*)a.ds_out + row * H + ch * 8, ds);
        float dx[8];
        if (drop) {
          float keep[8];
          dropout_mask8(dkey, row, H, ch * 8, dthr, keep);
#pragma unroll
          for (int j = 0; j < 8; ++j) dx[j] = ds[j] * keep[j] * keep_scale;
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) dx[j] = ds[j];
        }
        if (separate_dx) store_vec<T, 8>((T*)a.dx_out + row * H + ch * 8, dx);
        if (a.want_dbias)
#pragma unroll
          for (int j = 0; j < 8; ++j) pbi[c][j] += dx[j];
      }
    }
  }

  // Flush per-lane column partials: reduce the block's groups through LDS, then one
  // plain store per column of this block's [3, H] slab.
  for (int c = 0; c < C; ++c) {
    int ch = c * G + tid_in_group;
    __syncthreads();
    if (groups_per_block > 1) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        colbuf[0][threadIdx.x * 8 + j] = pg[c][j];
        colbuf[1][threadIdx.x * 8 + j] = pb[c][j];
        colbuf[2][threadIdx.x * 8 + j] = pbi[c][j];
      }
      __syncthreads();
      if (group == 0 && ch < nchunk) {
        for (int q = 1; q < groups_per_block; ++q) {
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            pg[c][j] += colbuf[0][(q * G + tid_in_group) * 8 + j];
            pb[c][j] += colbuf[1][(q * G + tid_in_group) * 8 + j];
            pbi[c][j] += colbuf[2][(q * G + tid_in_group) * 8 + j];
          }
        }
      }
    }
    if (group == 0 && ch < nchunk) {
      float* base = a.partials + (int64_t)blockIdx.x * 3 * H;
      store_vec<float, 8>(base + ch * 8, pg[c]);
      store_vec<float, 8>(base + H + ch * 8, pb[c]);
      store_vec<float, 8>(base + 2 * H + ch * 8, pbi[c]);
    }
  }
}

// Sum [nblocks, 3, H] partials into dgamma / dbeta / dbias (fp32 outputs).
__global__ __launch_bounds__(256) void ln_partials_reduce_kernel(const float* __restrict__ part,
                                                                int nblocks, int H,
                                                                float* __restrict__ dgamma,
                                                                float* __restrict__ dbeta,
                                                                float* __restrict__ dbias,
                                                                int acc_mask) {
  // blockIdx.y selects the quantity (slab rows have stride 3H); bit q of acc_mask = accumulate.
  const int q = blockIdx.y;
  float* out = q == 0 ? dgamma : (q == 1 ? dbeta : dbias);
  if (out == nullptr) return;
  colsum_block(part + (int64_t)q * H, nblocks, 3 * (int64_t)H, H, out, (acc_mask >> q) & 1);
}

template <typename T, typename W, int G>
static hipError_t ln_fwd_dispatch_c(const LnFwdArgs& a, int C, int grid, hipStream_t st) {
#define SMDT_LN_FWD_CASE(CC) \
  case CC: hipLaunchKernelGGL((ln_fwd_kernel<T, W, G, CC>), dim3(grid), dim3(256), 0, st, a); break;
  switch (C) {
    SMDT_LN_FWD_CASE(1) SMDT_LN_FWD_CASE(2) SMDT_LN_FWD_CASE(3) SMDT_LN_FWD_CASE(4)
    SMDT_LN_FWD_CASE(5) SMDT_LN_FWD_CASE(6) SMDT_LN_FWD_CASE(7) SMDT_LN_FWD_CASE(8)
    default: return hipErrorInvalidValue;
  }
#undef SMDT_LN_FWD_CASE
  return hipGetLastError();
}

template <typename T, typename W, int G>
static hipError_t ln_bwd_dispatch_c(const LnBwdArgs& a, int C, int grid, hipStream_t st) {
#define SMDT_LN_BWD_CASE(CC) \
  case CC: hipLaunchKernelGGL((ln_bwd_kernel<T, W, G, CC>), dim3(grid), dim3(256), 0, st, a); break;
  switch (C) {
    SMDT_LN_BWD_CASE(1) SMDT_LN_BWD_CASE(2) SMDT_LN_BWD_CASE(3) SMDT_LN_BWD_CASE(4)
    SMDT_LN_BWD_CASE(5) SMDT_LN_BWD_CASE(6) SMDT_LN_BWD_CASE(7) SMDT_LN_BWD_CASE(8)
    default: return hipErrorInvalidValue;
  }
#undef SMDT_LN_BWD_CASE
  return hipGetLastError();
}

// Row-group geometry: G threads per row and C 8-element chunks per thread.
static void ln_geometry(int H, int* G, int* C) {
  int nchunk = H / 8;
  if (H <= 2048) {
    *G = 64;
  } else {
    *G = 256;
  }
  *C = (nchunk + *G - 1) / *G;
}

template <typename T, typename W>
static hipError_t ln_fwd_typed(const LnFwdArgs& a, hipStream_t st) {
  int G, C;
  ln_geometry(a.H, &G, &C);
  int rows_per_block = 256 / G;
  int grid = stream_grid(a.rows, rows_per_block);
  if (G == 64) return ln_fwd_dispatch_c<T, W, 64>(a, C, grid, st);
  return ln_fwd_dispatch_c<T, W, 256>(a, C, grid, st);
}

template <typename T, typename W>
static hipError_t ln_bwd_typed(const LnBwdArgs& a, hipStream_t st) {
  int G, C;
  ln_geometry(a.H, &G, &C);
  if (G == 64) return ln_bwd_dispatch_c<T, W, 64>(a, C, a.nblocks, st);
  return ln_bwd_dispatch_c<T, W, 256>(a, C, a.nblocks, st);
}

}  // namespace smdt

using namespace smdt;

extern "C" int smdt_ln_bwd_nblocks(int64_t rows, int H) {
  int G, C;
  ln_geometry(H, &G, &C);
  int rows_per_block = 256 / G;
  int64_t b = (rows + rows_per_block - 1) / rows_per_block;
  // 512 blocks (2 per CU) keeps the fp32 partial slab small while filling the chip.
  if (b > 512) b = 512;
  if (b < 1) b = 1;
  return (int)b;
}

extern "C" hipError_t smdt_layernorm_fwd(int dtype, int wdtype, const void* x, const void* res,
                                         const void* bias, const void* gamma, const void* beta,
                                         void* y, void* s_out, float* mean, float* rstd,
                                         int64_t rows, int H, float eps, float p_drop,
                                         uint64_t seed, uint64_t offset, int rms,
                                         const void* x2, hipStream_t st) {
  if (H % 8 != 0 || H > 16384) return hipErrorInvalidValue;
  LnFwdArgs a{x, res, bias, gamma, beta, y, s_out, mean, rstd, rows, H, eps, p_drop, seed, offset, rms,
              smdt_rng_step(), x2};
  if (dtype == 1 && wdtype == 1) return ln_fwd_typed<bf16, bf16>(a, st);
  if (dtype == 1 && wdtype == 0) return ln_fwd_typed<bf16, float>(a, st);
  if (dtype == 2 && wdtype == 2) return ln_fwd_typed<f16, f16>(a, st);
  if (dtype == 2 && wdtype == 0) return ln_fwd_typed<f16, float>(a, st);
  if (dtype == 0 && wdtype == 0) return ln_fwd_typed<float, float>(a, st);
  return hipErrorInvalidValue;
}

extern "C" hipError_t smdt_layernorm_bwd(int dtype, int wdtype, const void* dy, const void* ds_in,
                                         const void* s, const void* gamma, const float* mean,
                                         const float* rstd, void* ds_out, void* dx_out,
                                         float* partials, int nblocks, float* dgamma,
                                         float* dbeta, float* dbias, int64_t rows, int H,
                                         float p_drop, uint64_t seed, uint64_t offset, int rms,
                                         int acc_mask, const void* dy2, hipStream_t st) {
  if (H % 8 != 0 || H > 16384) return hipErrorInvalidValue;
  LnBwdArgs a{dy, ds_in, s, gamma, mean, rstd, ds_out, dx_out, partials, rows, H, p_drop, seed,
              offset, rms, dbias != nullptr, nblocks, smdt_rng_step(), dy2};
  hipError_t e;
  if (dtype == 1 && wdtype == 1) e = ln_bwd_typed<bf16, bf16>(a, st);
  else if (dtype == 1 && wdtype == 0) e = ln_bwd_typed<bf16, float>(a, st);
  else if (dtype == 2 && wdtype == 2) e = ln_bwd_typed<f16, f16>(a, st);
  else if (dtype == 2 && wdtype == 0) e = ln_bwd_typed<f16, float>(a, st);
  else if (dtype == 0 && wdtype == 0) e = ln_bwd_typed<float, float>(a, st);
  else return hipErrorInvalidValue;
  if (e != hipSuccess) return e;
  dim3 grid((H + 31) / 32, 3);
  hipLaunchKernelGGL(ln_partials_reduce_kernel, grid, dim3(256), 0, st, partials, nblocks, H,
                     dgamma, rms ? nullptr : dbeta, dbias, acc_mask);
  return hipGetLastError();
}
