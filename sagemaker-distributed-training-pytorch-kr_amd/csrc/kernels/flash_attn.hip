// Flash attention (causal / full, MHA / GQA) forward and backward on gfx950 MFMA.
//
// The fused-attention path behind Megatron's `--use-flash-attn` flag
// (/root/reference/3_training_megatron-lm/megatron/arguments.py:825-827) and the
// MI355X replacement for the materialised [b*np, sq, sk] scores + K1 fused softmax path.
//
// Everything is built on `v_mfma_f32_32x32x16_bf16` (wave64, 32x32 output tile, K = 16) and on
// two gfx950 facts from the CDNA4 playbook (cdna_hip_programming.md §3, T10, T12):
//   * an MFMA accumulator tile X (column on the lane, rows in registers) can be fed, after a
//     bf16 pack, straight back as the B operand of a product that sums over X's ROW index
//     ("A·X"), provided the A operand uses the matching permuted k order;
//   * `ds_read_b64_tr_b16` delivers that permuted A operand (a column gather of 4 consecutive
//     rows) from a plain row-major LDS tile, so no transpose copy is ever made.
// Hence every kernel computes the "swapped" products so the softmax row index sits on the lane:
//   forward  : S^T = K.Q^T  (query on lane)  -> online softmax in registers -> O^T += V^T.P^T
//   dK/dV    : S   = Q.K^T  (key on lane)    -> dV^T += dO^T.P,  dK^T += Q^T.dS
//   dQ       : S^T = K.Q^T  (query on lane)  -> dQ^T += K^T.dS^T
// dK/dV and dQ run as two kernels (FA2 split) so there are no float atomics: deterministic
// results and no atomic-rate floor (HIP guide Guideline 12).
//
// v2 performance structure (measured VALU-bound in v1: 942 VALU vs 16 MFMA per tile):
//   * every LDS fragment address is a per-lane base computed ONCE plus a compile-time
//     immediate (the XOR swizzle only depends on row bits 0..3, so 16-row tile offsets are
//     constants) -> no address arithmetic inside the loops;
//   * softmax works in the log2 domain with raw `v_exp_f32` (__builtin_amdgcn_exp2f) and one
//     FMA per element; the row max / sum cross the two half-waves with v_permlane32_swap;
//   * the causal mask is applied only on the diagonal tile of each wave (uniform branch);
//   * K/V (resp. Q/dO) tiles are double-buffered in LDS with register staging issued before
//     the MFMA work of the current tile (T14), so each tile needs ONE barrier.
//
// LDS tiles are 64 rows x D bf16 with an XOR swizzle of the 16-byte chunk index that makes
// BOTH the row reads (ds_read_b128, 4x16-lane groups) and the transposed reads
// (ds_read_b64_tr_b16, 2x32-lane groups) bank-conflict free for D = 64 and D = 128.
//
// Layout: q/k/v/o are [B, S, heads, D] with arbitrary batch / token / head strides (elements),
// so the kernels read Q, K, V directly out of a fused QKV projection output. lse / delta are
// fp32 [B, H, S]. Requirements (checked by the launcher): S % 128 == 0, D in {64, 128},
// H % Hkv == 0, 16-byte aligned rows.
#include <cmath>

#include "common.h"
#include "launchers.h"
#include "mfma_tile.h"

namespace smdt {
namespace fa {

using namespace mt;
using s16x4 = mt::s16x4;

constexpr int kBlockRows = 128;  // rows owned by a workgroup (4 waves x 32)
// Block order. 1 (default): global longest-first. Block i runs row block i / (pairs) of the
// (b, h) pair i % (pairs), so every pair's heaviest causal block is dispatched first, then every
// pair's next-heaviest, and so on. The hardware deals blocks to the 8 XCDs round-robin, so with a
// pair count that is a multiple of 8 all row blocks of one (b, h) land on the SAME XCD, and its
// K / V (Q / dO in dK/dV) are re-read from that XCD's L2. 0: the (b, h)-major order (heaviest
// block first within each pair), which spreads one pair's blocks over all 8 L2s.
// Measured at B64 S1024 H16 D64 causal, dropout 0.1 (profiles/r2_attn_order/): fwd 0.426 ->
// 0.33-0.36 ms, bwd 1.29-1.31 -> 1.00-1.01 ms.
#ifndef SMDT_FA_ORDER
#define SMDT_FA_ORDER 1
#endif
constexpr float kLog2e = 1.4426950408889634f;

__device__ __forceinline__ float fexp2(float x) { return __builtin_amdgcn_exp2f(x); }

// max / sum of x with the value held by lane ^ 32 (same query / key, other half-wave).
__device__ __forceinline__ float xhalf_max(float x) {
  auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float xhalf_sum(float x) {
  auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

struct Strides {
  int64_t sb, ss, sh;
};

// Attention dropout. The 2x2 block (q, k), q, k in {2i, 2i+1} x {2j, 2j+1} shares one 32-bit
// hash of the block counter (q/2) * (S/2) + k/2 keyed by (seed, offset, b, h); byte
// 2 (q & 1) + (k & 1) of it decides the element: kept iff its low 7 bits >= T = round(p * 128)
// (kept probabilities scaled by inv = 128 / (128 - T)). The forward and both backward kernels
// re-derive the identical mask, no mask tensor is stored.
//
// VALU budget (the attention loops are VALU-issue-bound, profiles/r1_fa_glds): a lane needs only
// the 2 bytes of its row (column) of each block, and its neighbour lane (q ^ 1 or k ^ 1) needs the
// other 2 of the SAME words. So each lane hashes every other block, the pair swap the words by one
// DPP move, and a v_perm_b32 gathers the 4 bytes this lane needs into one word; the 4 threshold
// tests then run as ONE SWAR add ((w & 0x7F7F7F7F) + (128 - T) x 0x01010101: bit 7 + 8b is the
// decision of byte b), and the decisions land on packed 16-bit operand pairs with one
// v_pk_ashrrev_i16 per pair (sign bits 15 / 31 -> 0xFFFF / 0 halves) and one AND. Per element that
// is ~1/4 hash + ~1/2 masking instruction instead of 1/2 hash + 3 (extract, compare, select).
// The hash is a keyed two-round multiply/xor-shift mixer; Philox-7 would cost several times more
// VALU than the MFMA work of an attention tile on CDNA4.
struct Drop {
  uint32_t thr, key0, key1;
  // graph-safe RNG (smdt_set_rng_step): a device step counter mixed into every key at run time,
  // so a HIP graph replay draws new masks while the per-call (seed, offset) stays baked in
  const uint32_t* step;
  uint32_t k4;    // (128 - T) in every byte: the SWAR threshold addend
  float inv;      // 1 / (1 - p_realised)
  float keep;     // 1 - p_realised  (= 1 / inv)
  float log2inv;  // log2(inv): folded into the exponent so p' = p * inv costs nothing
};

__device__ __forceinline__ uint32_t fmix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x85EBCA6Bu;
  x ^= x >> 13;
  x *= 0xC2B2AE35u;
  x ^= x >> 16;
  return x;
}
__device__ __forceinline__ uint32_t drop_key(const Drop& d, int bh) {
  const uint32_t k = fmix32(d.key0 + (uint32_t)bh * 0x632BE5ABu) ^ d.key1;
  return d.step ? k ^ fmix32(*d.step * 0x9E3779B1u + 0x85EBCA77u) : k;
}
__device__ __forceinline__ uint32_t drop_hash(uint32_t blk, uint32_t key) {
  // full-rate ops only (v_mul_u32_u24, xor, shift): v_mul_lo_u32 is a quarter-rate instruction
  uint32_t x = blk ^ key;
  x = __umul24(x ^ (x >> 16), 0x45D9F3u);
  x = __umul24(x ^ (x >> 16), 0x45D9F3u);
  return x ^ (x >> 16);
}
// The partner lane's value (lane ^ 1): DPP quad_perm [1, 0, 3, 2].
__device__ __forceinline__ uint32_t swap_lane1(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xB1, 0xF, 0xF, true);
}
// Keep decisions of two slots (block words of slot 2u computed by the even lane, 2u + 1 by the odd
// one; ``h`` is this lane's word). ``sel`` (per lane) gathers [slot 2u lo, slot 2u+1 lo, slot 2u hi,
// slot 2u+1 hi] bytes; the result has the decision of that byte at bit 7 / 15 / 23 / 31.
__device__ __forceinline__ uint32_t keep_bits(uint32_t h, uint32_t sel, uint32_t k4) {
  const uint32_t w = __builtin_amdgcn_perm(h, swap_lane1(h), sel);
  return (w & 0x7F7F7F7Fu) + k4;
}
// 16-bit all-ones / zero halves from sign bits 15 / 31 (v_pk_ashrrev_i16).
__device__ __forceinline__ uint32_t half_masks(uint32_t t) {
  using s2 = __attribute__((ext_vector_type(2))) short;
  s2 v = __builtin_bit_cast(s2, t);
  v = v >> (short)15;
  return __builtin_bit_cast(uint32_t, v);
}
// Packed-pair masks of slot 2u (bits 7 / 23) and slot 2u + 1 (bits 15 / 31).
__device__ __forceinline__ uint32_t mask_even_slot(uint32_t t) { return half_masks(t << 8); }
__device__ __forceinline__ uint32_t mask_odd_slot(uint32_t t) { return half_masks(t); }
// keep bit b of t ? x : y with x, y fp32: v_bfe_i32 (all-ones / zero; only the bfe is asm, left to
// itself the compiler turns the sign-extend into test + compare + select) and ONE gfx950
// v_bitop3_b32 (LUT 0xCA = m ? x : y, bitwise) through its compiler-visible builtin, so the
// MFMA-result read of x stays inside the compiler's hazard padding. (The former
// (x & m) | (y & ~m) form compiled to three and / or instructions per element in these loops.)
template <int b>
__device__ __forceinline__ float sel_bit(float x, float y, uint32_t t) {
  int32_t m;
  asm("v_bfe_i32 %0, %1, %2, 1" : "=v"(m) : "v"(t), "n"(b));
  return __uint_as_float(__builtin_amdgcn_bitop3_b32((uint32_t)m, __float_as_uint(x), __float_as_uint(y), 0xCA));
}
// AND the four packed pairs of a 16-bit operand fragment with their masks.
template <class V>
__device__ __forceinline__ V and_pairs(V x, uint32_t m0, uint32_t m1, uint32_t m2, uint32_t m3) {
  using u4 = __attribute__((ext_vector_type(4))) uint32_t;
  u4 w = __builtin_bit_cast(u4, x);
  w[0] &= m0;
  w[1] &= m1;
  w[2] &= m2;
  w[3] &= m3;
  return __builtin_bit_cast(V, w);
}

// A row constant as an MFMA operand (see bwd_dq_kernel): lanes of half 0 hold x as three 16-bit
// terms in k-slots 0..2 (x - t0 - t1 - t2 below 2^-24 |x| for bf16), half 1 and the other slots 0;
// rowconst_ones is the matching all-ones operand.
template <class E>
__device__ __forceinline__ v8_t<E> rowconst_terms(float x, int h) {
  v8_t<E> v;
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = (E)0.f;
  if (h == 0) {
    const E t0 = (E)x;
    const float r1 = x - (float)t0;
    const E t1 = (E)r1;
    const E t2 = (E)(r1 - (float)t1);
    v[0] = t0;
    v[1] = t1;
    v[2] = t2;
  }
  return v;
}
// The dK / dV kernel's 16-byte row of BOTH constants: x's terms in k-slots 0..2, y's in 4..6, so
// one LDS row per query feeds both accumulator starts (rowconst_ones<E>(h, 0) picks x,
// rowconst_ones<E>(h, 4) picks y).
template <class E>
__device__ __forceinline__ v8_t<E> rowconst_pair(float x, float y) {
  const v8_t<E> a = rowconst_terms<E>(x, 0), c = rowconst_terms<E>(y, 0);
  v8_t<E> v = a;
#pragma unroll
  for (int j = 0; j < 3; ++j) v[4 + j] = c[j];
  return v;
}
template <class E>
__device__ __forceinline__ v8_t<E> rowconst_ones(int h, int first = 0) {
  v8_t<E> v;
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = (E)((h == 0 && j >= first && j < first + 3) ? 1.f : 0.f);
  return v;
}

// Operand prescale: x * c rounded back to bf16 (one-time, register-resident fragments).
template <class V>
__device__ __forceinline__ V scale8(V x, float c) {
  using EE = std::remove_cv_t<std::remove_reference_t<decltype(x[0])>>;
  V r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = (EE)((float)x[j] * c);
  return r;
}
// An opaque copy: keeps the compiler from hoisting a loop-invariant splat16 out of the tile
// loop (which pins 16 extra VGPRs per splat for the whole kernel).
__device__ __forceinline__ float opaque(float x) {
  float v;
  asm volatile("v_mov_b32 %0, %1" : "=v"(v) : "v"(x));
  return v;
}
__device__ __forceinline__ f32x16 splat16(float v) {
  f32x16 z;
#pragma unroll
  for (int i = 0; i < 16; ++i) z[i] = v;
  return z;
}

// Two exp2(x * c - b) values. Deliberately scalar v_fma_f32: packed v_pk_fma_f32 measured
// slower in these loops (it pins register pairs and is not faster per element on gfx950).
struct f2s {
  float x, y;
};
__device__ __forceinline__ f2s pexp2(float x0, float x1, float c, float b0, float b1) {
  return {fexp2(fmaf(x0, c, -b0)), fexp2(fmaf(x1, c, -b1))};
}

// s_waitcnt with vmcnt = n and the other counters left alone (gfx9 encoding).
template <int n>
__device__ __forceinline__ void wait_vm() {
  static_assert(n >= 0 && n < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((n & 15) | ((n >> 4) << 14) | (7 << 4) | (15 << 8));
}
using lds_void = __attribute__((address_space(3))) void;

// LDS-DMA of `bytes` per lane from a wave-uniform global base + a 32-bit per-lane byte offset,
// as buffer_load ... lds: the base lives in an SGPR buffer resource, the lane part in ONE VGPR
// (global_load_lds needs a 64-bit VGPR address per piece, kept live across the loop).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t dma_rsrc(const void* uniform_base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(uniform_base), (short)0, 0x7FFFFFFF, 0x00020000);
}
__device__ __forceinline__ void dma_lds16(const void* uniform_base, uint32_t voff, char* lds) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(dma_rsrc(uniform_base), (lds_void*)lds, 16, voff, 0, 0, 0);
}
__device__ __forceinline__ void dma_lds4(const void* uniform_base, uint32_t voff, char* lds) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(dma_rsrc(uniform_base), (lds_void*)lds, 4, voff, 0, 0, 0);
}

// This lane's index, re-made where it is used (2 VALU): asm volatile is never hoisted out of the
// tile loop, so a lane-derived DMA offset built from it holds no VGPR across the loop (the
// compiler spilled such loop-invariant offsets of the dK / dV kernel, and each scratch reload in
// the loop came with an s_waitcnt vmcnt(0) that drained the stage prefetch).
__device__ __forceinline__ uint32_t lane_now() {
  uint32_t l;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
  return l;
}

// LDS-DMA of one 64-row x D bf16 tile into its swizzled Geo<D> image: wave-instruction i writes
// 1 KB of LDS lane-linearly (rows 1024 / RB * i ..), so lane l lands at (row, slot l % CH) and
// loads the global chunk whose swizzled position that is: chunk slot ^ f(row).
template <int D>
struct GldsTile {
  static constexpr int kRowsPerInst = 1024 / Geo<D>::RB;             // 8 (D = 64) / 4 (D = 128)
  static constexpr int kPerWave = kTile * Geo<D>::RB / 1024 / 4;      // 2 / 4 per wave (4 waves)
  // BYTE offset of this lane's chunk from the tile's first row, unsigned 32-bit: with a
  // wave-uniform tile base the DMA then uses the SGPR-base + 32-bit VGPR-offset form (a signed /
  // 64-bit offset kept a VGPR pair per piece alive across the loop, and those were the values the
  // dK / dV kernel spilled and reloaded — each reload a vmcnt(0) that drained its own prefetch)
  uint32_t off[kPerWave];
  __device__ __forceinline__ void init(int w, int lane, int64_t row_stride) {
#pragma unroll
    for (int j = 0; j < kPerWave; ++j) {
      const int i = w * kPerWave + j;
      const int r = i * kRowsPerInst + lane / Geo<D>::CH;
      const int c = (lane % Geo<D>::CH) ^ Geo<D>::f(r);
      off[j] = (uint32_t)(r * row_stride + 8 * c) * 2u;
    }
  }
  template <class E>
  __device__ __forceinline__ void issue(const E* tile_base, char* img, int w) const {
#pragma unroll
    for (int j = 0; j < kPerWave; ++j) dma_lds16(tile_base, off[j], img + (w * kPerWave + j) * 1024);
  }
};

// ---------------------------------------------------------------------------------------
// Forward. Workgroup = 4 waves = 128 query rows of one (b, h); K/V streamed in 64-key tiles,
// double-buffered.
template <int D, bool CAUSAL, bool DROP, class E>
__global__ __launch_bounds__(256, D == 64 ? 2 : 1) void fwd_kernel(const E* __restrict__ Q,
                                                     const E* __restrict__ K,
                                                     const E* __restrict__ V,
                                                     E* __restrict__ O, float* __restrict__ LSE,
                                                     int B, int H, int Hkv, int S, Strides qs,
                                                     Strides ks_, Strides vs, Strides os,
                                                     float scale, Drop drop) {
  using G = Geo<D>;
  // Three [K | V] tile buffers (separate objects: the compiler sees that the LDS-DMA into one does
  // not alias the fragment reads of another, so it leaves the DMA queue alone).
  // D = 64: three [K | V] buffers, two tiles in flight; D = 128 (twice the bytes): two buffers,
  // so two workgroups still fit a CU's 160 KB of LDS.
  constexpr int kBuf = D == 64 ? 3 : 2;
  __shared__ __attribute__((aligned(16))) char L0[2 * G::TB], L1[2 * G::TB], L2[kBuf == 3 ? 2 * G::TB : 16];

  const int lane = threadIdx.x & 63, h = lane >> 5;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform: diagonal tests branch on SCC
  const int nqb = S / kBlockRows;
  // Heaviest (latest) causal blocks first: they have the most key tiles.
#if SMDT_FA_ORDER == 2
  // per XCD, pair-major: the row blocks of one (b, h) run together on one XCD, heaviest first
  const int nbh = gridDim.x / nqb;
  int qb, bh;
  if ((nbh & 7) == 0) {
    const int slot = blockIdx.x >> 3, r = slot % nqb;
    bh = (slot / nqb) * 8 + (blockIdx.x & 7);
    qb = CAUSAL ? nqb - 1 - r : r;
  } else {
    qb = CAUSAL ? (nqb - 1 - (int)(blockIdx.x / nbh)) : (int)(blockIdx.x / nbh);
    bh = blockIdx.x % nbh;
  }
#elif SMDT_FA_ORDER == 1
  // global longest-first: every (b, h)'s heaviest block, then the next-heaviest, ...
  const int nbh = gridDim.x / nqb;
  const int qb = CAUSAL ? (nqb - 1 - (int)(blockIdx.x / nbh)) : (int)(blockIdx.x / nbh);
  const int bh = blockIdx.x % nbh;
#else
  const int qb = CAUSAL ? (nqb - 1 - (int)(blockIdx.x % nqb)) : (int)(blockIdx.x % nqb);
  const int bh = blockIdx.x / nqb;
#endif
  const int b = bh / H, hq = bh % H, hk = hq / (H / Hkv);
  const int q0 = qb * kBlockRows;
  const int qw = q0 + 32 * w;  // this wave's first query row
  const int my_q = qw + (lane & 31);

  const E* Kb = K + b * ks_.sb + hk * ks_.sh;
  const E* Vb = V + b * vs.sb + hk * vs.sh;

  Frag<D, E> fr;
  fr.init(lane);
  v8_t<E> qf[G::KS];
  load_reg_frags<D>(Q + b * qs.sb + hq * qs.sh, qs.ss, qw, lane, qf);
  // Q is prescaled by scale * log2(e), so S^T comes out in the log2 domain, and the score
  // accumulator starts at -m (the reference max): p = exp2(S) needs no per-element FMA.
  const float c2 = scale * kLog2e;
#pragma unroll
  for (int kk = 0; kk < G::KS; ++kk) qf[kk] = scale8(qf[kk], c2);

  f32x16 o[G::DT];
#pragma unroll
  for (int t = 0; t < G::DT; ++t) o[t] = zero16();
  // Reference max m (log2 domain) starts at 0 and moves lazily (see below); l = denominator.
  float m = 0.f, l = 0.f;
  f32x16 negm = zero16();  // -m in all 16 registers: the score MFMAs' initial accumulator

  const int kend = CAUSAL ? (q0 + kBlockRows) : S;
  const int ntiles = kend / kTile;
  const uint32_t dkey = DROP ? drop_key(drop, bh) : 0u;
  const uint32_t shalf = (uint32_t)S >> 1;
  // block counter of this lane's first hashed key pair (key rows 4 h .. ; odd queries hash the
  // odd slots) and its byte gather: even q keeps bytes 0 / 1, odd q bytes 2 / 3
  const uint32_t dblk = (uint32_t)(my_q >> 1) * shalf + 2u * h + (uint32_t)(my_q & 1);
  const uint32_t dsel = (my_q & 1) ? 0x07030602u : 0x01050004u;
  // K/V tiles stream global -> LDS by LDS-DMA (global_load_lds, no VGPR staging, no ds_write
  // pass) through a 3-buffer ring with two tiles in flight: tile t waits only for its own DMA
  // (counted vmcnt) and one raw s_barrier publishes it.
  GldsTile<D> gk, gv;
  gk.init(w, lane, ks_.ss);
  gv.init(w, lane, vs.ss);
  auto issue = [&](int t, char* img) {
    gk.issue(Kb + (int64_t)t * kTile * ks_.ss, img, w);
    gv.issue(Vb + (int64_t)t * kTile * vs.ss, img + G::TB, w);
  };
  constexpr int kPer = 2 * GldsTile<D>::kPerWave;  // DMA wave-instructions per tile and wave
  issue(0, L0);
  if constexpr (kBuf == 3) issue(ntiles > 1 ? 1 : 0, L1);
  wait_vm<(kBuf - 2) * kPer>();
  __builtin_amdgcn_s_barrier();

  // Every call issues exactly one tile's DMA (past the end it re-reads the last tile into a
  // buffer nobody reads again), so the counted waits stay uniform.
  auto tile = [&](int t, const char* kt, char* pre) {
    const int kb = t * kTile;
    const char* vt = kt + G::TB;
    issue(t + kBuf - 1 < ntiles ? t + kBuf - 1 : ntiles - 1, pre);
    if (!CAUSAL || kb <= qw + 31) {
      // S^T tiles (log2 domain, minus m): rows = keys (registers), column = this lane's query.
      f32x16 st[2];
      auto scores = [&]() {
#pragma unroll
        for (int tt = 0; tt < 2; ++tt) {
          st[tt] = mfma(fr.rowf(kt, 32 * tt, 0), qf[0], negm);  // starts at -m: no per-tile splat
#pragma unroll
          for (int kk = 1; kk < G::KS; ++kk) st[tt] = mfma(fr.rowf(kt, 32 * tt, kk), qf[kk], st[tt]);
        }
        if (CAUSAL && kb + kTile - 1 > qw) {  // diagonal tile for this wave: mask key > query
          // kb is qw or qw - 32 (64-key tiles, 32-query waves): two lane-only patterns, so the
          // compares are loop-invariant and only the selects run, on diagonal tiles
          auto diag = [&](int off) {
#pragma unroll
            for (int tt = 0; tt < 2; ++tt)
#pragma unroll
              for (int i = 0; i < 16; ++i)
                if (off + 32 * tt + acc_row(i, h) > (lane & 31)) st[tt][i] = -INFINITY;
          };
          if (kb == qw) diag(0);
          else diag(-32);
        }
      };
      float rs0 = 0.f, rs1 = 0.f;  // two chains: the denominator uses the un-dropped p
      auto expsum = [&]() {
        rs0 = rs1 = 0.f;
#pragma unroll
        for (int tt = 0; tt < 2; ++tt)
#pragma unroll
          for (int i = 0; i < 16; i += 2) {
            const float p0 = fexp2(st[tt][i]), p1 = fexp2(st[tt][i + 1]);
            rs0 += p0;
            rs1 += p1;
            st[tt][i] = p0;
            st[tt][i + 1] = p1;
          }
        return xhalf_sum(rs0 + rs1);
      };
      scores();
      // Lazy reference max without a per-tile row max: p = exp2(S - m) is taken straight away and
      // m only moves when the row's tile sum leaves [2^-64, 2^64] (p that large or small is still
      // exact in fp32 / bf16, l and O have range to spare) — too large (or not finite), or, before
      // anything was accumulated, so small that the row could underflow. Wave-uniform branch
      // (ballot); rare: it recomputes the tile's scores (the K tile is still in LDS), takes the
      // exact row max, rescales and redoes the exponentials. Saves the ~21 max instructions per
      // tile of a per-tile max (the loop is VALU-issue-bound).
      float rsum = expsum();
      const bool bad = !(rsum <= 0x1p64f) || (l == 0.f && rsum < 0x1p-64f);
      if (__builtin_amdgcn_ballot_w64(bad) != 0) {
        scores();
        float tmax = st[0][0];
#pragma unroll
        for (int tt = 0; tt < 2; ++tt)
#pragma unroll
          for (int i = 0; i < 16; ++i) tmax = fmaxf(tmax, st[tt][i]);
        tmax = xhalf_max(tmax);
        const float d = bad ? tmax : 0.f;
        const float alpha = fexp2(-d);
        l *= alpha;
#pragma unroll
        for (int dt = 0; dt < G::DT; ++dt) o[dt] *= alpha;
#pragma unroll
        for (int tt = 0; tt < 2; ++tt) st[tt] -= d;
        m += d;
        negm = splat16(-m);
        rsum = expsum();
      }
      // dropout: packed-pair masks of the 8 key-pair slots of each 32-key sub-tile (slot m =
      // registers 2m, 2m + 1); dropped entries leave P.V only (l sums the un-dropped p) and the
      // 1/(1-p) scale is applied in the epilogue
      uint32_t dm[2][8];
      if constexpr (DROP) {
#pragma unroll
        for (int tt = 0; tt < 2; ++tt)
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const uint32_t t = keep_bits(drop_hash(dblk + ((kb + 32 * tt) >> 1) + 4 * u, dkey), dsel, drop.k4);
            dm[tt][2 * u] = mask_even_slot(t);
            dm[tt][2 * u + 1] = mask_odd_slot(t);
          }
      }
      l += rsum;
      // O^T[d, q] += V^T[d, keys] . P^T[keys, q]
#pragma unroll
      for (int tt = 0; tt < 2; ++tt) {
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          v8_t<E> pb = pack8<E>(st[tt], s);
          if constexpr (DROP) pb = and_pairs(pb, dm[tt][4 * s], dm[tt][4 * s + 1], dm[tt][4 * s + 2], dm[tt][4 * s + 3]);
#pragma unroll
          for (int dt = 0; dt < G::DT; ++dt) o[dt] = mfma(fr.trf(vt, 32 * tt, s, dt), pb, o[dt]);
        }
      }
    }
    wait_vm<(kBuf - 2) * kPer>();  // tile t + 1 landed (t + 2 may still be in flight)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  };
  if constexpr (kBuf == 3) {
    for (int t = 0; t < ntiles; t += 3) {
      tile(t, L0, L2);
      if (t + 1 < ntiles) tile(t + 1, L1, L0);
      if (t + 2 < ntiles) tile(t + 2, L2, L1);
    }
  } else {
    for (int t = 0; t < ntiles; t += 2) {
      tile(t, L0, L1);
      if (t + 1 < ntiles) tile(t + 1, L1, L0);
    }
  }
  wait_vm<0>();  // drain the trailing re-read before the workgroup's LDS is released

  // Epilogue: O[q, d] = O^T / l (x 1/(1-p) with dropout) ; lse = (m + log2 l) * ln 2.
  const float inv = l > 0.f ? (DROP ? drop.inv : 1.f) / l : 0.f;
  E* Ob = O + b * os.sb + hq * os.sh + (int64_t)my_q * os.ss;
#pragma unroll
  for (int dt = 0; dt < G::DT; ++dt) {
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      v4_t<E> v4;
#pragma unroll
      for (int j = 0; j < 4; ++j) v4[j] = (E)(o[dt][4 * g + j] * inv);
      *reinterpret_cast<v4_t<E>*>(Ob + 32 * dt + 8 * g + 4 * h) = v4;
    }
  }
  if (h == 0) LSE[((int64_t)b * H + hq) * S + my_q] = (m + __log2f(l)) * 0.6931471805599453f;
}

// ---------------------------------------------------------------------------------------
// The backward kernels' per-query row constants, ready to be loaded straight into MFMA
// accumulators (no VALU in their loops):
//   ndl[b, h, q]   = -keep * sum_d dO[q, d] O[q, d]      (-delta', the dP accumulator's start)
//   nlse2[b, h, q] = -(lse log2 e - log2 inv)           (the S accumulator's start, log2 domain)
// They are made by the dQ kernel, which runs first and holds dO of its query rows in registers
// anyway (one extra read of O's rows); the dK / dV kernel reads them from memory. (Round 3 had a
// separate streaming delta kernel: 1.6 ms per GPT-2 345M step)

// ---------------------------------------------------------------------------------------
// dK / dV. Workgroup = 4 waves = 128 keys of one (b, kv-head); each wave keeps K, V of its 32
// keys and dK^T, dV^T in registers while the workgroup sweeps the query heads of the group and
// their 64-row query tiles (Q, dO, lse*log2e, delta staged in double-buffered LDS).
// Workgroups per CU requested from the compiler for the D = 64 backward kernels (A/B knobs).
#ifndef SMDT_FA_DQ_OCC
#define SMDT_FA_DQ_OCC 2
#endif
#ifndef SMDT_FA_DQ_BUF
#define SMDT_FA_DQ_BUF 3   // K / V stage slots of the D = 64 dQ kernel
#endif
// dQ: re-make the two accumulator splats (-lse', -delta') per 32-key sub-tile instead of pinning
// them for the whole kernel: 178 -> 140 VGPRs, 2 -> 3 waves per SIMD, no spills; measured bwd
// 1.014 / 1.041 -> 0.991 / 1.004 ms at B64 (profiles/r2_attn_order/ab_b64_dq_remat.log).
#ifndef SMDT_FA_DQ_REMAT
#define SMDT_FA_DQ_REMAT 2
#endif
#ifndef SMDT_FA_DKDV_ROLLED
#define SMDT_FA_DKDV_ROLLED 0
#endif
// The two row constants share one 16-byte LDS row per query: 52,992 B of LDS per workgroup, so
// three workgroups would fit a CU (56,064 B before). Asking the compiler for 3 (168 VGPRs) spills
// 140 B per lane in the dropout variant and measured 605 vs 564 us per call at the bench shape
// (profiles/r5_dkdv_occ/): the kernel stays at 2 workgroups per CU.
#ifndef SMDT_FA_DKDV_OCC
#define SMDT_FA_DKDV_OCC 2
#endif
template <int D, bool CAUSAL, bool DROP, class E>
__global__ __launch_bounds__(256, D == 64 ? SMDT_FA_DKDV_OCC : 1) void bwd_dkdv_kernel(
    const E* __restrict__ Q, const E* __restrict__ K, const E* __restrict__ V,
    const E* __restrict__ dO, const E* __restrict__ RC3,
    const float* __restrict__ DELTA, E* __restrict__ dK, E* __restrict__ dV, int B, int H, int Hkv, int S,
    Strides qs, Strides ks_, Strides vs, Strides dos, Strides dks, Strides dvs, float scale, Drop drop) {
  using G = Geo<D>;
  using VF = v8_t<E>;
  // Q | dO | the tile's 64 query rows of the row constants as ONE 16-bit term row each (16 B,
  // written by the dQ kernel: -(lse log2e - log2 inv) in k-slots 0..2, -delta' in 4..6) | -delta'
  // fp32 (dropout only)
  constexpr int kRC = kTile * 16;
  constexpr int RCB = kRC + kTile * 4;
  // D = 64: three stage slots, two work items in flight; D = 128: two (LDS budget). Q, dO and the
  // row constants of a slot are SEPARATE __shared__ objects: with one object per slot the compiler
  // drained the DMA queue (s_waitcnt vmcnt(0)) between the Q and the dO pieces of every item,
  // i.e. it waited for the prefetch it had just issued (round-3 listing); the forward kernel's
  // K | V slots had no such drain.
  constexpr int kBuf = D == 64 ? 3 : 2;
  __shared__ __attribute__((aligned(16))) char Q0[G::TB], Q1[G::TB], Q2[kBuf == 3 ? G::TB : 16];
  __shared__ __attribute__((aligned(16))) char O0[G::TB], O1[G::TB], O2[kBuf == 3 ? G::TB : 16];
  __shared__ __attribute__((aligned(16))) char R0[RCB], R1[RCB], R2[kBuf == 3 ? RCB : 16];
  auto qbuf = [&](int sl) -> char* { return sl == 0 ? Q0 : sl == 1 ? Q1 : Q2; };
  auto obuf = [&](int sl) -> char* { return sl == 0 ? O0 : sl == 1 ? O1 : O2; };
  auto rbuf = [&](int sl) -> char* { return sl == 0 ? R0 : sl == 1 ? R1 : R2; };

  const int lane = threadIdx.x & 63, h = lane >> 5;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform: diagonal tests branch on SCC
  const int nkb = S / kBlockRows;
#if SMDT_FA_ORDER == 2
  const int nbhk = gridDim.x / nkb;
  int kblk, bhk;
  if ((nbhk & 7) == 0) {
    const int slot = blockIdx.x >> 3;
    kblk = slot % nkb;
    bhk = (slot / nkb) * 8 + (blockIdx.x & 7);
  } else {
    kblk = (int)(blockIdx.x / nbhk);
    bhk = blockIdx.x % nbhk;
  }
#elif SMDT_FA_ORDER == 1
  const int nbhk = gridDim.x / nkb;
  const int kblk = (int)(blockIdx.x / nbhk);  // global longest-first
  const int bhk = blockIdx.x % nbhk;
#else
  const int kblk = (int)(blockIdx.x % nkb);  // early key blocks see the most query tiles
  const int bhk = blockIdx.x / nkb;
#endif
  const int b = bhk / Hkv, hk = bhk % Hkv;
  const int group = H / Hkv;
  const int k0 = kblk * kBlockRows;
  const int kw = k0 + 32 * w;
  const int my_key = kw + (lane & 31);

  Frag<D, E> fr;
  fr.init(lane);
  v8_t<E> kf[G::KS], vf[G::KS];
  load_reg_frags<D>(K + b * ks_.sb + hk * ks_.sh, ks_.ss, kw, lane, kf);
  load_reg_frags<D>(V + b * vs.sb + hk * vs.sh, vs.ss, kw, lane, vf);
  const VF ones_l = rowconst_ones<E>(h, 0), ones_d = rowconst_ones<E>(h, 4);
#pragma unroll
  for (int kk = 0; kk < G::KS; ++kk) kf[kk] = scale8(kf[kk], scale * kLog2e);  // S in log2 domain

  f32x16 dk[G::DT], dv[G::DT];
#pragma unroll
  for (int t = 0; t < G::DT; ++t) dk[t] = dv[t] = zero16();
  const float c2 = scale * kLog2e;

  const int qstart = CAUSAL ? k0 : 0;
  const int ntiles = (S - qstart) / kTile;
  const int total = ntiles * group;

  // Q / dO tiles and the tile's raw lse / delta rows stream in by LDS-DMA through a ring of kBuf
  // stage buffers (waves 0 / 1 also move the 64 lse / 64 delta floats of the tile). Work items
  // (query head, query tile) advance as running counters: no integer division in the loop.
  GldsTile<D> gq, gdo;
  gq.init(w, lane, qs.ss);
  gdo.init(w, lane, dos.ss);
  constexpr int kPer = 2 * GldsTile<D>::kPerWave;
  int ih_n = 0, iq_n = 0, issued = 0;  // next work item to stream in
  auto issue = [&](int sl) {
    // every call issues one item's DMA (past the end: the last item again, into a slot nobody
    // reads), so the counted waits stay uniform
    const int ih = issued < total ? ih_n : group - 1, iq = issued < total ? iq_n : ntiles - 1;
    const int hq = hk * group + ih;
    const int qb = qstart + iq * kTile;
    gq.issue(Q + b * qs.sb + hq * qs.sh + (int64_t)qb * qs.ss, qbuf(sl), w);
    gdo.issue(dO + b * dos.sb + hq * dos.sh + (int64_t)qb * dos.ss, obuf(sl), w);
    const int64_t r0 = ((int64_t)b * H + hq) * S + qb;
    if (w == 0) {
      dma_lds16(RC3 + r0 * 8, lane_now() << 4, rbuf(sl));
    } else if (DROP && w == 1) {
      dma_lds4(DELTA + r0, lane_now() << 2, rbuf(sl) + kRC);
    }
    ++issued;
    if (++iq_n == ntiles) {
      iq_n = 0;
      ++ih_n;
    }
  };
  auto wait_next = [&]() {  // the next item's DMA has landed (a later one may still be in flight)
    if (w == 0 || (DROP && w == 1)) wait_vm<(kBuf - 2) * (kPer + 1)>();
    else wait_vm<(kBuf - 2) * kPer>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  };
  issue(0);
  if constexpr (kBuf == 3) issue(1);
  wait_next();

  const uint32_t shalf = (uint32_t)S >> 1;
  // even keys keep bytes 0 / 2 of each block word, odd keys bytes 1 / 3; odd keys hash odd slots
  const uint32_t dsel = (my_key & 1) ? 0x07030501u : 0x02060004u;
  // Causal mask as part of the S accumulator's initial value: a wave's 32 x 32 (query, key) block
  // is either fully visible, fully masked (skipped) or exactly its diagonal block (qsub == kw),
  // whose pattern (key > query) is the same for every diagonal block: there the initial value is
  // -1e30 where this lane's key follows register i's query, so no compare / select runs after the
  // exponential (exp2(-1e30) = 0). Only the diagonal items build that pattern (sd_init), so it
  // holds no registers in the main loop.
  int ch = 0, cq = 0;  // current work item
  auto item = [&](int cur, int pre) {
    const int qb = qstart + cq * kTile;
    const uint32_t dkey = DROP ? drop_key(drop, b * H + hk * group + ch) : 0u;
    const uint32_t dblk = ((uint32_t)((qb + 4 * h) >> 1) + (uint32_t)(my_key & 1)) * shalf + (uint32_t)(my_key >> 1);
    const char* q_l = qbuf(cur);
    const char* do_l = obuf(cur);
    const char* rc_l = rbuf(cur);
    const float* del_l = reinterpret_cast<const float*>(rc_l + kRC);
    issue(pre);
    // S'[q, key] = Q . K'^T - lse ; dP'[q, key] = dO . V^T - delta  (key on lane, query rows in
    // registers). The row constants enter as one MFMA k-step ahead of each chain (A = the query
    // row's three 16-bit terms from LDS, B = ones in k-slots 0..2; half 1's A values meet B's
    // zeros): no accumulator moves. The causal diagonal block masks key > query after the chain.
    auto sd_init = [&](int qs2, f32x16& sa, f32x16& pa) {
      const int r = 32 * qs2 + (lane & 31);
      const VF rc = *reinterpret_cast<const VF*>(rc_l + 16 * r);
      sa = mfma(rc, ones_l, zero16());
      pa = mfma(rc, ones_d, zero16());
    };
    auto diag_mask = [&](f32x16& sa) {
#pragma unroll
      for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if ((lane & 31) > 8 * g + 4 * h + j) sa[4 * g + j] = -1e30f;
    };
    auto sd_mma = [&](int qs2, f32x16& sa, f32x16& pa) {
#pragma unroll
      for (int kk = 0; kk < G::KS; ++kk) {
        sa = mfma(fr.rowf(q_l, 32 * qs2, kk), kf[kk], sa);
        pa = mfma(fr.rowf(do_l, 32 * qs2, kk), vf[kk], pa);
      }
    };
    // P' = exp2(S') and dS = P' (dP - delta') -> 16-bit operands. Dropout: slot m = registers
    // 2m, 2m + 1 (queries 2i, 2i + 1 of one block); dropped entries: P' -> 0 for dV (packed-pair
    // masks), dP -> 0, so dS = p' (keep ? dP : 0) - p' delta'.
    auto softmax_ds = [&](int qs2, f32x16& sa, f32x16& pa, v8_t<E> (&pb)[2], v8_t<E> (&db)[2]) {
      uint32_t dm[8];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int r0 = 32 * qs2 + 8 * g + 4 * h;
        const f32x4 ndl = DROP ? *reinterpret_cast<const f32x4*>(del_l + r0) : f32x4{0.f, 0.f, 0.f, 0.f};
        uint32_t t = 0u;
        if constexpr (DROP) {
          t = keep_bits(drop_hash(dblk + (uint32_t)(16 * qs2 + 4 * g) * shalf, dkey), dsel, drop.k4);
          dm[2 * g] = mask_even_slot(t);
          dm[2 * g + 1] = mask_odd_slot(t);
        }
#pragma unroll
        for (int j = 0; j < 4; j += 2) {
          const int i = 4 * g + j;
          // with dropout: p / (1 - p_drop); 0 where the causal mask was folded into s
          const float p0 = fexp2(sa[i]), p1 = fexp2(sa[i + 1]);
          float d0 = pa[i], d1 = pa[i + 1];
          if constexpr (DROP) {  // kept: dP - delta'; dropped: -delta'
            if (j == 0) {
              d0 = sel_bit<7>(d0, ndl[j], t);
              d1 = sel_bit<23>(d1, ndl[j + 1], t);
            } else {
              d0 = sel_bit<15>(d0, ndl[j], t);
              d1 = sel_bit<31>(d1, ndl[j + 1], t);
            }
          }
          sa[i] = p0;
          sa[i + 1] = p1;
          pa[i] = p0 * d0;  // dS
          pa[i + 1] = p1 * d1;
        }
      }
#pragma unroll
      for (int st = 0; st < 2; ++st) {
        pb[st] = pack8<E>(sa, st);
        if constexpr (DROP) pb[st] = and_pairs(pb[st], dm[4 * st], dm[4 * st + 1], dm[4 * st + 2], dm[4 * st + 3]);
        db[st] = pack8<E>(pa, st);
      }
    };
    // dV^T[d, key] += dO^T[d, q] . P[q, key] ; dK^T[d, key] += Q^T[d, q] . dS[q, key]
    auto acc_mma = [&](int qs2, const v8_t<E> (&pb)[2], const v8_t<E> (&db)[2]) {
#pragma unroll
      for (int st = 0; st < 2; ++st)
#pragma unroll
        for (int dt = 0; dt < G::DT; ++dt) {
          dv[dt] = mfma(fr.trf(do_l, 32 * qs2, st, dt), pb[st], dv[dt]);
          dk[dt] = mfma(fr.trf(q_l, 32 * qs2, st, dt), db[st], dk[dt]);
        }
    };
    // ONE code path for every item: the two 32-query halves one after the other (48 fewer live
    // VGPRs than straight-line code, which spilled at 256 VGPRs once the row constants entered as
    // MFMA operands; the partner wave on the SIMD supplies the overlap of softmax VALU and MFMAs).
    // Causal items only add wave-uniform tests: a half whose queries all precede this wave's keys
    // is skipped, the diagonal half masks key > query. (A separate straight path for the
    // non-diagonal items made the compiler keep dK / dV in two register sets and copy all 64
    // accumulator VGPRs, 64 v_mov_b64, on every item's loop back-edge.)
#pragma unroll
    for (int qs2 = 0; qs2 < 2; ++qs2) {
      const int qsub = qb + 32 * qs2;
      if (CAUSAL && qsub + 31 < kw) continue;  // all queries precede all of this wave's keys
      f32x16 sa, pa;
      v8_t<E> pb[2], db[2];
      sd_init(qs2, sa, pa);
      sd_mma(qs2, sa, pa);
      if (CAUSAL && qsub == kw) diag_mask(sa);  // the diagonal block: key > query is masked
      softmax_ds(qs2, sa, pa, pb, db);
      acc_mma(qs2, pb, db);
    }
    if (++cq == ntiles) {
      cq = 0;
      ++ch;
    }
    wait_next();
  };
#if SMDT_FA_DKDV_ROLLED
  // One work item per iteration, the stage slots rotating as wave-uniform counters (their LDS
  // bases are selected per item, SALU): the unrolled kBuf-item body with a conditional call per
  // item made the compiler copy the dK / dV accumulators (32 v_mov_b64) on the joins.
  {
    int cur = 0, pre = kBuf - 1;
#pragma nounroll
    for (int it = 0; it < total; ++it) {
      item(cur, pre);
      cur = cur + 1 == kBuf ? 0 : cur + 1;
      pre = pre + 1 == kBuf ? 0 : pre + 1;
    }
  }
#else
  if constexpr (kBuf == 3) {
    for (int it = 0; it < total; it += 3) {
      item(0, 2);
      if (it + 1 < total) item(1, 0);
      if (it + 2 < total) item(2, 1);
    }
  } else {
    for (int it = 0; it < total; it += 2) {
      item(0, 1);
      if (it + 1 < total) item(1, 0);
    }
  }
#endif
  wait_vm<0>();  // drain the trailing re-reads before the workgroup's LDS is released


  // dK[key, d] = scale * dK^T ; dV[key, d] = dV^T (key on lane, d in registers)
  E* dKb = dK + b * dks.sb + hk * dks.sh + (int64_t)my_key * dks.ss;
  E* dVb = dV + b * dvs.sb + hk * dvs.sh + (int64_t)my_key * dvs.ss;
#pragma unroll
  for (int dt = 0; dt < G::DT; ++dt) {
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      v4_t<E> a, c;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        a[j] = (E)(dk[dt][4 * g + j] * scale);
        c[j] = (E)dv[dt][4 * g + j];
      }
      *reinterpret_cast<v4_t<E>*>(dKb + 32 * dt + 8 * g + 4 * h) = a;
      *reinterpret_cast<v4_t<E>*>(dVb + 32 * dt + 8 * g + 4 * h) = c;
    }
  }
}

// ---------------------------------------------------------------------------------------
// dQ. Workgroup = 4 waves = 128 query rows of one (b, h); K/V streamed in 64-key tiles,
// double-buffered.
template <int D, bool CAUSAL, bool DROP, class E>
__global__ __launch_bounds__(256, D == 64 ? SMDT_FA_DQ_OCC : 1) void bwd_dq_kernel(
    const E* __restrict__ Q, const E* __restrict__ K, const E* __restrict__ V,
    const E* __restrict__ dO, const E* __restrict__ O, const float* __restrict__ LSE,
    float* __restrict__ DELTA, E* __restrict__ RC3, E* __restrict__ dQ, int B, int H, int Hkv,
    int S, Strides qs, Strides ks_, Strides vs, Strides dos, Strides os, Strides dqs, float scale,
    float dscale, float lsub, Drop drop) {
  using G = Geo<D>;
  // D = 64: three [K | V] buffers, two tiles in flight; D = 128 (twice the bytes): two buffers,
  // so two workgroups still fit a CU's 160 KB of LDS.
  constexpr int kBuf = D == 64 ? SMDT_FA_DQ_BUF : 2;
  __shared__ __attribute__((aligned(16))) char L0[2 * G::TB], L1[2 * G::TB], L2[kBuf == 3 ? 2 * G::TB : 16];

  const int lane = threadIdx.x & 63, h = lane >> 5;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform: diagonal tests branch on SCC
  const int nqb = S / kBlockRows;
#if SMDT_FA_ORDER == 2
  // per XCD, pair-major: the row blocks of one (b, h) run together on one XCD, heaviest first
  const int nbh = gridDim.x / nqb;
  int qb, bh;
  if ((nbh & 7) == 0) {
    const int slot = blockIdx.x >> 3, r = slot % nqb;
    bh = (slot / nqb) * 8 + (blockIdx.x & 7);
    qb = CAUSAL ? nqb - 1 - r : r;
  } else {
    qb = CAUSAL ? (nqb - 1 - (int)(blockIdx.x / nbh)) : (int)(blockIdx.x / nbh);
    bh = blockIdx.x % nbh;
  }
#elif SMDT_FA_ORDER == 1
  // global longest-first: every (b, h)'s heaviest block, then the next-heaviest, ...
  const int nbh = gridDim.x / nqb;
  const int qb = CAUSAL ? (nqb - 1 - (int)(blockIdx.x / nbh)) : (int)(blockIdx.x / nbh);
  const int bh = blockIdx.x % nbh;
#else
  const int qb = CAUSAL ? (nqb - 1 - (int)(blockIdx.x % nqb)) : (int)(blockIdx.x % nqb);
  const int bh = blockIdx.x / nqb;
#endif
  const int b = bh / H, hq = bh % H, hk = hq / (H / Hkv);
  const int q0 = qb * kBlockRows;
  const int qw = q0 + 32 * w;
  const int my_q = qw + (lane & 31);

  Frag<D, E> fr;
  fr.init(lane);
  v8_t<E> qf[G::KS], dof[G::KS];
  load_reg_frags<D>(Q + b * qs.sb + hq * qs.sh, qs.ss, qw, lane, qf);
  load_reg_frags<D>(dO + b * dos.sb + hq * dos.sh, dos.ss, qw, lane, dof);
#pragma unroll
  for (int kk = 0; kk < G::KS; ++kk) qf[kk] = scale8(qf[kk], scale * kLog2e);  // S^T in log2 domain
  // Row constants -(lse log2e - log2 inv) and -delta' = -keep sum_d dO O, made here from this
  // lane's dO fragments (lanes l and l ^ 32 hold the two 8-column halves of every 16 columns of
  // the row) and stored for the dK / dV kernel, which runs next; they are the S / dP MFMAs'
  // initial accumulators.
  const int64_t ridx = ((int64_t)b * H + hq) * S + my_q;
  float ndl;
  {
    v8_t<E> of[G::KS];
    load_reg_frags<D>(O + b * os.sb + hq * os.sh, os.ss, qw, lane, of);
    float acc = 0.f;
#pragma unroll
    for (int kk = 0; kk < G::KS; ++kk)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc = fmaf((float)of[kk][j], (float)dof[kk][j], acc);
    ndl = -xhalf_sum(acc) * dscale;
  }
  const float nlse2 = lsub - LSE[ridx] * kLog2e;
  if (h == 0) {   // for the dK / dV kernel: fp32 -delta' (dropout path) and both in one term row
    DELTA[ridx] = ndl;
    *reinterpret_cast<v8_t<E>*>(RC3 + ridx * 8) = rowconst_pair<E>(nlse2, ndl);
  }
#if SMDT_FA_DQ_REMAT == 2
  // The row constants enter as one extra MFMA k-step per chain: A = 1 in k-slots 0..2 of every
  // key row, B = the constant of this lane's query split into three 16-bit terms (t0 + t1 + t2
  // carries ~24 bits of it), so S' / dP' start at c = 1.t0 + 1.t1 + 1.t2 without the 2 x 16 VALU
  // moves of a per-sub-tile splat and without pinning 32 VGPRs for a resident one: the loops are
  // VALU-issue-bound (scripts/isa_loop_stats.py), the matrix pipe has room.
  const v8_t<E> ones3 = rowconst_ones<E>(h);
  const v8_t<E> lse3 = rowconst_terms<E>(nlse2, h), dl3 = rowconst_terms<E>(ndl, h);
#define SMDT_DQ_ST0 mfma(ones3, lse3, zero16())
#define SMDT_DQ_DP0 mfma(ones3, dl3, zero16())
#elif SMDT_FA_DQ_REMAT
  // the two accumulator splats are re-made per sub-tile (opaque: not hoisted), freeing 32 VGPRs
#define SMDT_DQ_ST0 splat16(opaque(nlse2))
#define SMDT_DQ_DP0 splat16(opaque(ndl))
#else
  const f32x16 st0 = splat16(nlse2), dp0 = splat16(ndl);  // dP' = dP - delta' (dropout selects below)
#define SMDT_DQ_ST0 st0
#define SMDT_DQ_DP0 dp0
#endif
  const float c2 = scale * kLog2e;
  const uint32_t dkey = DROP ? drop_key(drop, bh) : 0u;
  const uint32_t dblk = (uint32_t)(my_q >> 1) * ((uint32_t)S >> 1) + 2u * h + (uint32_t)(my_q & 1);
  const uint32_t dsel = (my_q & 1) ? 0x07030602u : 0x01050004u;

  const E* Kb = K + b * ks_.sb + hk * ks_.sh;
  const E* Vb = V + b * vs.sb + hk * vs.sh;

  f32x16 dq[G::DT];
#pragma unroll
  for (int t = 0; t < G::DT; ++t) dq[t] = zero16();

  const int kend = CAUSAL ? (q0 + kBlockRows) : S;
  const int ntiles = kend / kTile;
  // K/V tiles by LDS-DMA through a 3-buffer ring, two tiles in flight (as in the forward).
  GldsTile<D> gk, gv;
  gk.init(w, lane, ks_.ss);
  gv.init(w, lane, vs.ss);
  auto issue = [&](int t, char* img) {
    gk.issue(Kb + (int64_t)t * kTile * ks_.ss, img, w);
    gv.issue(Vb + (int64_t)t * kTile * vs.ss, img + G::TB, w);
  };
  constexpr int kPer = 2 * GldsTile<D>::kPerWave;
  issue(0, L0);
  if constexpr (kBuf == 3) issue(ntiles > 1 ? 1 : 0, L1);
  wait_vm<(kBuf - 2) * kPer>();
  __builtin_amdgcn_s_barrier();

  auto tile = [&](int t, const char* kt, char* pre) {
    const int kb = t * kTile;
    const char* vt = kt + G::TB;
    issue(t + kBuf - 1 < ntiles ? t + kBuf - 1 : ntiles - 1, pre);
    // row constants as the initial accumulators: S' = S log2(e) scale - lse, dP' = dP - delta
    auto sd = [&](int tt, f32x16& st, f32x16& dpt) {
      st = mfma(fr.rowf(kt, 32 * tt, 0), qf[0], SMDT_DQ_ST0);
      dpt = mfma(fr.rowf(vt, 32 * tt, 0), dof[0], SMDT_DQ_DP0);
#pragma unroll
      for (int kk = 1; kk < G::KS; ++kk) {
        st = mfma(fr.rowf(kt, 32 * tt, kk), qf[kk], st);
        dpt = mfma(fr.rowf(vt, 32 * tt, kk), dof[kk], dpt);
      }
    };
    // causal diagonal sub-tile: key > query gets S' = -1e30 (exp2 -> 0), ONE uniform block before
    // the softmax. (Testing it per element pair inside the softmax made the compiler branch on the
    // flag around every pair: 16 basic blocks per sub-tile, no MFMA / VALU interleave across them.)
    auto diag_mask = [&](int tt, f32x16& st) {
      const int ksub = kb + 32 * tt;
#pragma unroll
      for (int i = 0; i < 16; ++i)
        if (ksub + acc_row(i, h) > my_q) st[i] = -1e30f;
    };
    // dS^T into dpt (P' = exp2(S'); dropout: kept dP - delta', dropped -delta')
    auto soft = [&](int tt, const f32x16& st, f32x16& dpt) {
      const int ksub = kb + 32 * tt;
      uint32_t tb[4];  // keep bits of slots 2u (bits 7 / 23) and 2u + 1 (bits 15 / 31)
      if constexpr (DROP) {
#pragma unroll
        for (int u = 0; u < 4; ++u) tb[u] = keep_bits(drop_hash(dblk + (ksub >> 1) + 4 * u, dkey), dsel, drop.k4);
      }
#pragma unroll
      for (int i = 0; i < 16; i += 2) {
        const float p0 = fexp2(st[i]), p1 = fexp2(st[i + 1]);  // with dropout: p / (1 - p_drop)
        float d0 = dpt[i], d1 = dpt[i + 1];
        if constexpr (DROP) {
          const uint32_t tw = tb[i >> 2];
          if ((i & 2) == 0) {
            d0 = sel_bit<7>(d0, ndl, tw);
            d1 = sel_bit<23>(d1, ndl, tw);
          } else {
            d0 = sel_bit<15>(d0, ndl, tw);
            d1 = sel_bit<31>(d1, ndl, tw);
          }
        }
        dpt[i] = p0 * d0;
        dpt[i + 1] = p1 * d1;
      }
    };
    // dQ^T[d, q] += K^T[d, keys] . dS^T[keys, q]
    auto acc = [&](int tt, const f32x16& dpt) {
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const v8_t<E> db = pack8<E>(dpt, s);
#pragma unroll
        for (int dt = 0; dt < G::DT; ++dt) dq[dt] = mfma(fr.trf(kt, 32 * tt, s, dt), db, dq[dt]);
      }
    };
    // (a straight-line pair of the two sub-tiles measured neutral, profiles/r4_attn_dq_straight_neutral/)
#pragma unroll
    for (int tt = 0; tt < 2; ++tt) {
      const int ksub = kb + 32 * tt;
      if (CAUSAL && ksub > qw + 31) continue;
      f32x16 st, dpt;
      sd(tt, st, dpt);
      if (CAUSAL && ksub + 31 > qw) diag_mask(tt, st);
      soft(tt, st, dpt);
      acc(tt, dpt);
    }
    wait_vm<(kBuf - 2) * kPer>();  // tile t + 1 landed (t + 2 may still be in flight)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  };
  if constexpr (kBuf == 3) {
    for (int t = 0; t < ntiles; t += 3) {
      tile(t, L0, L2);
      if (t + 1 < ntiles) tile(t + 1, L1, L0);
      if (t + 2 < ntiles) tile(t + 2, L2, L1);
    }
  } else {
    for (int t = 0; t < ntiles; t += 2) {
      tile(t, L0, L1);
      if (t + 1 < ntiles) tile(t + 1, L1, L0);
    }
  }
  wait_vm<0>();

  E* dQb = dQ + b * dqs.sb + hq * dqs.sh + (int64_t)my_q * dqs.ss;
#pragma unroll
  for (int dt = 0; dt < G::DT; ++dt) {
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      v4_t<E> a;
#pragma unroll
      for (int j = 0; j < 4; ++j) a[j] = (E)(dq[dt][4 * g + j] * scale);
      *reinterpret_cast<v4_t<E>*>(dQb + 32 * dt + 8 * g + 4 * h) = a;
    }
  }
}

}  // namespace fa
}  // namespace smdt

using namespace smdt;
using namespace smdt::fa;

static bool fa_shape_ok(int dtype, int H, int Hkv, int S, int D) {
  return (dtype == 1 || dtype == 2) && (D == 64 || D == 128) && S % kBlockRows == 0 && S > 0 && S <= 65536 &&
         Hkv > 0 && H % Hkv == 0;
}

static uint32_t host_fmix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x85EBCA6Bu;
  x ^= x >> 13;
  x *= 0xC2B2AE35u;
  x ^= x >> 16;
  return x;
}

static uint32_t* g_rng_step = nullptr;
extern "C" void smdt_set_rng_step(uint32_t* counter) { g_rng_step = counter; }
extern "C" uint32_t* smdt_rng_step() { return g_rng_step; }

// keys: key0 from the seed, key1 from the per-call offset (see drop_key / drop_hash).
static Drop make_drop(float p, uint64_t seed, uint64_t offset) {
  Drop d;
  d.thr = (uint32_t)((double)p * 128.0 + 0.5);  // 7-bit threshold (SWAR test, see Drop)
  if (d.thr > 127u) d.thr = 127u;
  d.k4 = (128u - d.thr) * 0x01010101u;
  d.inv = (float)(128.0 / (128.0 - (double)d.thr));  // exact for the realised drop rate
  d.keep = (float)((128.0 - (double)d.thr) / 128.0);
  d.log2inv = (float)std::log2(128.0 / (128.0 - (double)d.thr));
  d.key0 = host_fmix32((uint32_t)seed ^ host_fmix32((uint32_t)(seed >> 32) + 0x9E3779B9u));
  d.key1 = host_fmix32((uint32_t)offset * 0x27D4EB2Fu ^ host_fmix32((uint32_t)(offset >> 32) + 0x165667B1u));
  d.step = smdt_rng_step();
  return d;
}

extern "C" hipError_t smdt_flash_fwd(int dtype, const void* q, const void* k, const void* v,
                                     void* o, float* lse, int B, int H, int Hkv, int S, int D,
                                     int64_t q_sb, int64_t q_ss, int64_t q_sh, int64_t k_sb,
                                     int64_t k_ss, int64_t k_sh, int64_t v_sb, int64_t v_ss,
                                     int64_t v_sh, int64_t o_sb, int64_t o_ss, int64_t o_sh,
                                     float scale, int causal, float dropout_p, uint64_t seed,
                                     uint64_t offset, hipStream_t st) {
  if (!fa_shape_ok(dtype, H, Hkv, S, D) || dropout_p < 0.f || dropout_p >= 1.f) return hipErrorInvalidValue;
  Strides qs{q_sb, q_ss, q_sh}, ks{k_sb, k_ss, k_sh}, vs{v_sb, v_ss, v_sh}, os{o_sb, o_ss, o_sh};
  dim3 grid((unsigned)((int64_t)B * H * (S / kBlockRows)));
  const Drop dr = make_drop(dropout_p, seed, offset);
  const bool drop = dropout_p > 0.f;
#define SMDT_FA_FWD(DD, CC, DR)                                                                 \
  do {                                                                                          \
    if (dtype == 2)                                                                             \
      hipLaunchKernelGGL((fwd_kernel<DD, CC, DR, f16>), grid, dim3(256), 0, st, (const f16*)q,  \
                         (const f16*)k, (const f16*)v, (f16*)o, lse, B, H, Hkv, S, qs, ks, vs, os, \
                         scale, dr);                                                            \
    else                                                                                        \
      hipLaunchKernelGGL((fwd_kernel<DD, CC, DR, bf16>), grid, dim3(256), 0, st, (const bf16*)q, \
                         (const bf16*)k, (const bf16*)v, (bf16*)o, lse, B, H, Hkv, S, qs, ks, vs, os, \
                         scale, dr);                                                            \
  } while (0)
#define SMDT_FA_FWD2(DD, CC) \
  do { if (drop) SMDT_FA_FWD(DD, CC, true); else SMDT_FA_FWD(DD, CC, false); } while (0)
  if (D == 64) { if (causal) SMDT_FA_FWD2(64, true); else SMDT_FA_FWD2(64, false); }
  else { if (causal) SMDT_FA_FWD2(128, true); else SMDT_FA_FWD2(128, false); }
#undef SMDT_FA_FWD2
#undef SMDT_FA_FWD
  return hipGetLastError();
}

extern "C" hipError_t smdt_flash_bwd(int dtype, const void* q, const void* k, const void* v,
                                     const void* o, const void* dout, const float* lse,
                                     float* delta, void* dq, void* dk, void* dv, int B, int H,
                                     int Hkv, int S, int D, const int64_t* strides, float scale,
                                     int causal, float dropout_p, uint64_t seed, uint64_t offset,
                                     hipStream_t st) {
  if (!fa_shape_ok(dtype, H, Hkv, S, D) || dropout_p < 0.f || dropout_p >= 1.f) return hipErrorInvalidValue;
  const Drop dr = make_drop(dropout_p, seed, offset);
  const bool drop = dropout_p > 0.f;
  // strides: 8 x (batch, seq, head) element strides for q, k, v, o, dO, dQ, dK, dV.
  Strides qs{strides[0], strides[1], strides[2]}, ks{strides[3], strides[4], strides[5]},
      vs{strides[6], strides[7], strides[8]}, os{strides[9], strides[10], strides[11]},
      dos{strides[12], strides[13], strides[14]}, dqs{strides[15], strides[16], strides[17]},
      dks{strides[18], strides[19], strides[20]}, dvs{strides[21], strides[22], strides[23]};
  // delta holds 10 x [B, H, S] fp32 words, written by the dQ kernel (which therefore runs first)
  // and read by the dK / dV kernel: -delta' rows, then (after one unused [B, H, S] slot) the
  // 16-byte term rows of -(lse log2e - log2 inv) and -delta' (see rowconst_pair)
  const int64_t bhs = (int64_t)B * H * S;
  void* rc3 = delta + 2 * bhs;
  const float dscale = drop ? dr.keep : 1.f, lsub = drop ? dr.log2inv : 0.f;
  dim3 gkv((unsigned)((int64_t)B * Hkv * (S / kBlockRows)));
  dim3 gq((unsigned)((int64_t)B * H * (S / kBlockRows)));
#define SMDT_FA_BWD_T(DD, CC, DR, ET)                                                            \
  do {                                                                                           \
    hipLaunchKernelGGL((bwd_dq_kernel<DD, CC, DR, ET>), gq, dim3(256), 0, st, (const ET*)q,      \
                       (const ET*)k, (const ET*)v, (const ET*)dout, (const ET*)o, lse, delta,     \
                       (ET*)rc3, (ET*)dq, B, H, Hkv, S, qs, ks, vs, dos, os, dqs,                 \
                       scale, dscale, lsub, dr);                                                  \
    hipLaunchKernelGGL((bwd_dkdv_kernel<DD, CC, DR, ET>), gkv, dim3(256), 0, st, (const ET*)q,  \
                       (const ET*)k, (const ET*)v, (const ET*)dout, (const ET*)rc3, delta,        \
                       (ET*)dk, (ET*)dv, B, H, Hkv, S, qs, ks, vs, dos, dks, dvs, scale, dr);     \
  } while (0)
#define SMDT_FA_BWD(DD, CC, DR) \
  do { if (dtype == 2) SMDT_FA_BWD_T(DD, CC, DR, f16); else SMDT_FA_BWD_T(DD, CC, DR, bf16); } while (0)
#define SMDT_FA_BWD2(DD, CC) \
  do { if (drop) SMDT_FA_BWD(DD, CC, true); else SMDT_FA_BWD(DD, CC, false); } while (0)
  if (D == 64) { if (causal) SMDT_FA_BWD2(64, true); else SMDT_FA_BWD2(64, false); }
  else { if (causal) SMDT_FA_BWD2(128, true); else SMDT_FA_BWD2(128, false); }
#undef SMDT_FA_BWD2
#undef SMDT_FA_BWD
#undef SMDT_FA_BWD_T
  return hipGetLastError();
}
