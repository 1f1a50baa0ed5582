// Shared device helpers for the gfx950 (CDNA4 / MI355X) kernel library.
//
// Everything here is written for wave64 CDNA4 directly: lane masks are 64-bit,
// reductions run over 64 lanes, and bf16 conversion relies on the native
// `__bf16` type, which hipcc lowers to v_cvt_pk_bf16_f32 on gfx950.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <type_traits>

namespace smdt {

constexpr int kWave = 64;

using bf16 = __bf16;
using f16 = _Float16;

// 16-byte vector of 8 x 16-bit elements (one global_load_dwordx4 per lane).
using u16x8 = __attribute__((ext_vector_type(8))) unsigned short;
using f32x4 = __attribute__((ext_vector_type(4))) float;
using f32x16 = __attribute__((ext_vector_type(16))) float;
using bf16x8 = __attribute__((ext_vector_type(8))) __bf16;
using i16x8 = __attribute__((ext_vector_type(8))) short;

enum class DType : int { kF32 = 0, kBF16 = 1, kF16 = 2 };

__device__ __forceinline__ float to_f32(float x) { return x; }
__device__ __forceinline__ float to_f32(bf16 x) { return (float)x; }
__device__ __forceinline__ float to_f32(f16 x) { return (float)x; }

template <typename T> __device__ __forceinline__ T from_f32(float x);
template <> __device__ __forceinline__ float from_f32<float>(float x) { return x; }
template <> __device__ __forceinline__ bf16 from_f32<bf16>(float x) { return (bf16)x; }
template <> __device__ __forceinline__ f16 from_f32<f16>(float x) { return (f16)x; }

// Vectorised load/store of N contiguous elements into/out of fp32 registers.
// N * sizeof(T) is 16 bytes for the 16-bit types with N = 8 and for fp32 with
// N = 4; larger N is issued as several 16-byte accesses.
// NT = true: nontemporal (streaming) loads for data a kernel reads exactly once.
template <typename T, int N, bool NT = false>
__device__ __forceinline__ void load_vec(const T* __restrict__ p, float (&out)[N]) {
  if constexpr (sizeof(T) == 2) {
    static_assert(N % 8 == 0, "16-bit vector loads move 8 elements");
#pragma unroll
    for (int c = 0; c < N / 8; ++c) {
      u16x8 v = NT ? __builtin_nontemporal_load(reinterpret_cast<const u16x8*>(p + c * 8))
                   : *reinterpret_cast<const u16x8*>(p + c * 8);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        unsigned short bits = v[j];
        T t;
        __builtin_memcpy(&t, &bits, 2);
        out[c * 8 + j] = to_f32(t);
      }
    }
  } else {
    static_assert(N % 4 == 0, "fp32 vector loads move 4 elements");
#pragma unroll
    for (int c = 0; c < N / 4; ++c) {
      f32x4 v = NT ? __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(p + c * 4))
                   : *reinterpret_cast<const f32x4*>(p + c * 4);
#pragma unroll
      for (int j = 0; j < 4; ++j) out[c * 4 + j] = v[j];
    }
  }
}

template <typename T, int N>
__device__ __forceinline__ void store_vec(T* __restrict__ p, const float (&in)[N]) {
  if constexpr (sizeof(T) == 2) {
    static_assert(N % 8 == 0, "16-bit vector stores move 8 elements");
#pragma unroll
    for (int c = 0; c < N / 8; ++c) {
      u16x8 v;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        T t = from_f32<T>(in[c * 8 + j]);
        unsigned short bits;
        __builtin_memcpy(&bits, &t, 2);
        v[j] = bits;
      }
      *reinterpret_cast<u16x8*>(p + c * 8) = v;
    }
  } else {
    static_assert(N % 4 == 0, "fp32 vector stores move 4 elements");
#pragma unroll
    for (int c = 0; c < N / 4; ++c) {
      f32x4 v;
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = in[c * 4 + j];
      *reinterpret_cast<f32x4*>(p + c * 4) = v;
    }
  }
}

// Elements per 16-byte access for T.
template <typename T> constexpr int vec_elems() { return 16 / (int)sizeof(T); }

// 8 elements of T kept in their raw (unconverted) form: one 16-byte register quad for 16-bit T,
// two for fp32. Lets a kernel issue the next row's loads before converting the current row's
// (software pipelining without paying the fp32 registers of the prefetched data).
using u32x4 = __attribute__((ext_vector_type(4))) unsigned;
template <typename T>
struct Raw8 {
  u32x4 v[sizeof(T) / 2];
};
template <typename T>
__device__ __forceinline__ Raw8<T> load_raw8(const T* __restrict__ p) {
  Raw8<T> r;
#pragma unroll
  for (int i = 0; i < (int)(sizeof(T) / 2); ++i) r.v[i] = reinterpret_cast<const u32x4*>(p)[i];
  return r;
}
// Streaming (nontemporal) forms for data touched exactly once per kernel: `nt` keeps the lines out
// of the way of other traffic in L2 (MI355X_MICROARCH.md: nt loads are L2-served at the plain
// rate; nt stores keep the line in the XCD's L2 like plain ones).
template <typename T>
__device__ __forceinline__ Raw8<T> load_raw8_nt(const T* __restrict__ p) {
  Raw8<T> r;
#pragma unroll
  for (int i = 0; i < (int)(sizeof(T) / 2); ++i) r.v[i] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p) + i);
  return r;
}
template <typename T>
__device__ __forceinline__ void store_vec8_nt(T* __restrict__ p, const float (&in)[8]) {
  static_assert(sizeof(T) == 2, "16-bit element streams");
  u16x8 v;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    T t = from_f32<T>(in[j]);
    unsigned short bits;
    __builtin_memcpy(&bits, &t, 2);
    v[j] = bits;
  }
  __builtin_nontemporal_store(v, reinterpret_cast<u16x8*>(p));
}
template <typename T>
__device__ __forceinline__ void cvt_raw8(const Raw8<T>& r, float (&out)[8]) {
  if constexpr (sizeof(T) == 2) {
    const u16x8 v = __builtin_bit_cast(u16x8, r.v[0]);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const unsigned short bits = v[j];
      T t;
      __builtin_memcpy(&t, &bits, 2);
      out[j] = to_f32(t);
    }
  } else {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const f32x4 f = __builtin_bit_cast(f32x4, r.v[i]);
#pragma unroll
      for (int j = 0; j < 4; ++j) out[4 * i + j] = f[j];
    }
  }
}

// ---------------------------------------------------------------------------
// wave64 reductions. __shfl_xor lowers to DPP / ds_swizzle / ds_bpermute as the
// compiler sees fit; all 64 lanes participate.
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, kWave));
  return v;
}

// Block-wide sum for a block of `nwaves` waves. `scratch` holds >= nwaves floats.
__device__ __forceinline__ float block_sum(float v, float* scratch, int nwaves) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  v = wave_sum(v);
  if (lane == 0) scratch[wid] = v;
  __syncthreads();
  float r = (lane < nwaves) ? scratch[lane] : 0.f;
  r = wave_sum(r);
  __syncthreads();
  return r;
}
__device__ __forceinline__ float block_max(float v, float* scratch, int nwaves) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  v = wave_max(v);
  if (lane == 0) scratch[wid] = v;
  __syncthreads();
  float r = (lane < nwaves) ? scratch[lane] : -INFINITY;
  r = wave_max(r);
  __syncthreads();
  return r;
}

// ---------------------------------------------------------------------------
// Counter-based RNG (Philox-4x32-7). Stateless: the random word for
// (seed, offset, idx) is the same in the forward and the backward kernel, so
// dropout masks are recomputed instead of stored.
__device__ __forceinline__ uint4 philox4x32(uint2 key, uint4 ctr) {
  constexpr uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
  constexpr uint32_t W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
  for (int r = 0; r < 7; ++r) {
    uint32_t hi0 = __umulhi(M0, ctr.x), lo0 = M0 * ctr.x;
    uint32_t hi1 = __umulhi(M1, ctr.z), lo1 = M1 * ctr.z;
    ctr = make_uint4(hi1 ^ ctr.y ^ key.x, lo1, hi0 ^ ctr.w ^ key.y, lo0);
    key.x += W0;
    key.y += W1;
  }
  return ctr;
}

// Four uniform floats in [0, 1) for counter `idx` (each call covers 4 elements).
__device__ __forceinline__ void philox_uniform4(uint64_t seed, uint64_t offset, uint64_t idx,
                                                float (&u)[4]) {
  uint2 key = make_uint2((uint32_t)seed, (uint32_t)(seed >> 32));
  uint4 ctr = make_uint4((uint32_t)idx, (uint32_t)(idx >> 32), (uint32_t)offset,
                         (uint32_t)(offset >> 32));
  uint4 r = philox4x32(key, ctr);
  constexpr float kInv = 2.3283064365386963e-10f;  // 2^-32
  u[0] = r.x * kInv;
  u[1] = r.y * kInv;
  u[2] = r.z * kInv;
  u[3] = r.w * kInv;
}

// Column sums of an fp32 [nrows, ncols] slab with row stride `rs` (the second stage of every
// "per-block partials" reduction: dgamma / dbeta / dbias). Block = 256 threads arranged as
// 32 columns x 8 row groups (128-byte coalesced row segments, 8x more loads in flight than a
// thread-per-column loop); the 8 group sums are combined in a fixed order (deterministic).
// Launch with grid.x = ceil(ncols / 32).
// out[col] (=|+=) sum_r part[r * rs + col]; accumulate=true adds into an existing fp32 buffer
// (e.g. a DDP main_grad), so no separate cast/add pass is needed.
__device__ __forceinline__ void colsum_block(const float* __restrict__ part, int nrows, int64_t rs,
                                             int ncols, float* __restrict__ out, bool accumulate = false) {
  __shared__ float red[8][33];
  const int cl = threadIdx.x & 31, rg = threadIdx.x >> 5;
  const int col = blockIdx.x * 32 + cl;
  // 16 independent chains, all 16 loads of a round issued before any add: the partial slabs are
  // a few MB and the kernel is latency-bound (512 rows = 4 dependent rounds per lane instead of
  // 16 with 4 chains: 7.5 -> 5.5 us per call at 8 chains, profiles/r5_colsum/)
  constexpr int NCH = 16;
  float a[NCH];
#pragma unroll
  for (int k = 0; k < NCH; ++k) a[k] = 0.f;
  if (col < ncols) {
    int r = rg;
    for (; r + 8 * (NCH - 1) < nrows; r += 8 * NCH) {
      float v[NCH];
#pragma unroll
      for (int k = 0; k < NCH; ++k) v[k] = part[(int64_t)(r + 8 * k) * rs + col];
#pragma unroll
      for (int k = 0; k < NCH; ++k) a[k] += v[k];
    }
    for (; r < nrows; r += 8) a[0] += part[(int64_t)r * rs + col];
  }
#pragma unroll
  for (int w = NCH / 2; w > 0; w /= 2)
#pragma unroll
    for (int k = 0; k < w; ++k) a[k] += a[k + w];
  red[rg][cl] = a[0];
  __syncthreads();
  if (rg == 0 && col < ncols) {
    float s = 0.f;
#pragma unroll
    for (int g = 0; g < 8; ++g) s += red[g][cl];
    out[col] = accumulate ? out[col] + s : s;
  }
}

// Number of blocks for a grid-stride memory-bound kernel (Guideline 11:
// cap at ~8 blocks per CU over 256 CUs).
inline int stream_grid(int64_t work_items, int per_block) {
  int64_t b = (work_items + per_block - 1) / per_block;
  if (b > 2048) b = 2048;
  if (b < 1) b = 1;
  return (int)b;
}

}  // namespace smdt
