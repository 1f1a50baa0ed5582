// Shared MFMA tile machinery for gfx950 kernels that stream 64-row bf16 tiles through LDS and
// read them both by rows (ds_read_b128) and by columns (ds_read_b64_tr_b16): the flash-attention
// kernels and the weight-gradient GEMM.
//
//   * v_mfma_f32_32x32x16_bf16: lane l holds A[i = l & 31][k = 8 (l >> 5) + j] and
//     B[k = 8 (l >> 5) + j][n = l & 31]; the 32x32 f32 result lands as
//     D[row = (r & 3) + 8 (r >> 2) + 4 (l >> 5)][col = l & 31] in register r (acc_row).
//   * Geo<D>: a 64-row x D-col bf16 LDS tile with an XOR swizzle of the 16-byte chunk index
//     (depends on row bits 0..3 only) that keeps BOTH the row reads and the transposed reads
//     bank-conflict free for D = 64 / 128.
//   * Frag<D>::trf returns the A-operand fragment of tile COLUMN 32 dt + (l & 31) over 16 tile
//     rows (rbase + 16 s + a fixed permutation). The permutation depends only on the lane half,
//     so two trf fragments of tiles with the same row structure also pair as (A, B) operands of
//     a product that sums over the tile ROWS (A^T . B with both operands row-major).
#pragma once
#include "common.h"

namespace smdt {
namespace mt {

using s16x4 = __attribute__((ext_vector_type(4))) short;
using s16x8 = __attribute__((ext_vector_type(8))) short;
using lds_s16x4 = __attribute__((address_space(3))) s16x4;
using bf4 = __attribute__((ext_vector_type(4))) __bf16;
using f16x8 = __attribute__((ext_vector_type(8))) _Float16;
using h4 = __attribute__((ext_vector_type(4))) _Float16;

// Element type -> MFMA operand vector (8 elements) and 4-element store vector. Both 16-bit types
// share every LDS layout and DMA path; only the MFMA opcode and the fp32 -> 16-bit rounding differ.
template <class E> struct Vec;
template <> struct Vec<bf16> { using v8 = bf16x8; using v4 = bf4; };
template <> struct Vec<f16> { using v8 = f16x8; using v4 = h4; };
template <class E> using v8_t = typename Vec<E>::v8;
template <class E> using v4_t = typename Vec<E>::v4;

constexpr int kTile = 64;        // rows per streamed LDS tile

__device__ __forceinline__ f32x16 mfma(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
// fp16 operands (Megatron --fp16): v_mfma_f32_32x32x16_f16, same lane / register maps.
__device__ __forceinline__ f32x16 mfma(f16x8 a, f16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ f32x16 zero16() {
  f32x16 z;
#pragma unroll
  for (int i = 0; i < 16; ++i) z[i] = 0.f;
  return z;
}

template <int D>
struct Geo {
  static constexpr int RB = D * 2;             // bytes per tile row
  static constexpr int TB = kTile * RB;        // bytes per tile
  static constexpr int KS = D / 16;            // MFMA k-steps over D
  static constexpr int DT = D / 32;            // 32-wide d tiles
  static constexpr int CH = D / 8;             // 16-byte chunks per row
  // Swizzle: depends on row bits 0..3 only, so offsets of rows r and r + 16 k differ by a
  // constant.
  __device__ static __forceinline__ int f(int r) {
    if constexpr (D >= 128) return ((r & 3) << 2) | ((r >> 2) & 3);
    else return (((r >> 1) & 1) << 2) | ((r >> 2) & 3);
  }
  __device__ static __forceinline__ int off(int r, int c) { return r * RB + 16 * (c ^ f(r)); }
};

// Per-lane LDS offsets, computed once per kernel. E = element type of the tiles.
template <int D, class E = bf16>
struct Frag {
  using V = v8_t<E>;
  int row[D / 16];     // row fragment of k-step ks for tile rows 0..31
  int tr[D / 32][2];   // transposed fragment of d-tile dt, k-step 0, rows 0..15 (two 4-row blocks)
  // Offset of the transposed read of d-tile dt, 4-row block `blk` (rows 4 h + (lane >> 2 & 3) + 8 blk).
  __device__ static __forceinline__ int tr_off(int lane, int dt, int blk) {
    const int h = lane >> 5, q = (lane >> 2) & 3, p = lane & 3, g = (lane >> 4) & 1;
    return Geo<D>::off(4 * h + q + 8 * blk, 4 * dt + 2 * g + (p >> 1)) + 8 * (p & 1);
  }
  __device__ __forceinline__ void init(int lane) {
    const int l31 = lane & 31, h = lane >> 5;
#pragma unroll
    for (int ks = 0; ks < D / 16; ++ks) row[ks] = Geo<D>::off(l31, 2 * ks + h);
#pragma unroll
    for (int dt = 0; dt < D / 32; ++dt) {
      tr[dt][0] = tr_off(lane, dt, 0);
      tr[dt][1] = tr_off(lane, dt, 1);
    }
  }
  // Transposed fragment at precomputed offsets (o0, o1) = (tr_off(.., 0), tr_off(.., 1)).
  __device__ static __forceinline__ V trf_at(const char* tile, int rbase, int s, int o0, int o1) {
    const char* b = tile + (rbase + 16 * s) * Geo<D>::RB;
    s16x4 x = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(b + o0));
    s16x4 y = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(b + o1));
    return __builtin_bit_cast(V, __builtin_shufflevector(x, y, 0, 1, 2, 3, 4, 5, 6, 7));
  }
  // A-operand row fragment: rows rbase..rbase+31 (rbase multiple of 32), elements 16 ks + 8 h..
  __device__ __forceinline__ V rowf(const char* tile, int rbase, int ks) const {
    return *reinterpret_cast<const V*>(tile + rbase * Geo<D>::RB + row[ks]);
  }
  // A-operand transposed fragment over tile rows rbase + 16 s + (permuted), columns 32 dt + lane&31.
  __device__ __forceinline__ V trf(const char* tile, int rbase, int s, int dt) const {
    return trf_at(tile, rbase, s, tr[dt][0], tr[dt][1]);
  }
};

// Pack accumulator registers 8 s .. 8 s + 7 into a 16-bit operand fragment.
template <class E = bf16>
__device__ __forceinline__ v8_t<E> pack8(const f32x16& x, int s) {
  v8_t<E> r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = (E)x[8 * s + j];
  return r;
}

// Row of accumulator register i for lane half h (32x32 C/D map).
__device__ __forceinline__ int acc_row(int i, int h) { return (i & 3) + 8 * (i >> 2) + 4 * h; }

// Global -> register staging of a 64-row tile (256 threads, 16-byte chunks).
template <int D>
struct Stage {
  static constexpr int N = kTile * Geo<D>::CH / 256;
  u16x8 v[N];
  int lds_off[N];
  int64_t goff[N];     // element offset of chunk i relative to the tile's first row
  int rowi[N];
  __device__ __forceinline__ void init(int64_t row_stride) {
#pragma unroll
    for (int i = 0; i < N; ++i) {
      const int idx = threadIdx.x + 256 * i;
      const int r = idx / Geo<D>::CH, c = idx % Geo<D>::CH;
      rowi[i] = r;
      lds_off[i] = Geo<D>::off(r, c);
      goff[i] = (int64_t)r * row_stride + c * 8;
    }
  }
  __device__ __forceinline__ void load(const bf16* tile_base) {
#pragma unroll
    for (int i = 0; i < N; ++i) v[i] = *reinterpret_cast<const u16x8*>(tile_base + goff[i]);
  }
  __device__ __forceinline__ void store(char* tile) const {
#pragma unroll
    for (int i = 0; i < N; ++i) *reinterpret_cast<u16x8*>(tile + lds_off[i]) = v[i];
  }
};

// Direct global load of a row-operand fragment that stays in registers for the whole kernel:
// lane holds row (row0 + lane&31), elements [16 ks + 8 h, +8).
template <int D, class E>
__device__ __forceinline__ void load_reg_frags(const E* base, int64_t row_stride, int row0,
                                               int lane, v8_t<E> (&f)[D / 16]) {
  const E* p = base + (int64_t)(row0 + (lane & 31)) * row_stride + 8 * (lane >> 5);
#pragma unroll
  for (int ks = 0; ks < D / 16; ++ks) f[ks] = *reinterpret_cast<const v8_t<E>*>(p + 16 * ks);
}


}  // namespace mt
}  // namespace smdt
