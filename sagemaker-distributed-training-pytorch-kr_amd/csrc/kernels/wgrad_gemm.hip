// Weight-gradient GEMM with fp32 accumulation into the DDP main_grad:
//     C[n, k] (fp32) += sum_m A[m, n] * B[m, k]       A = dY [M, N], B = X [M, K], bf16 / fp16 row-major
// (Megatron's gradient-accumulation fusion; /root/reference/3_training_megatron-lm/
// megatron/arguments.py:850-854).
//
// Why a hand-written kernel: the reduction index m (tokens) is the SLOW index of both operands.
// Library GEMMs treat that as the "NT" layout and stage each operand through an LDS transpose;
// gfx950's ds_read_b64_tr_b16 reads a row-major [m][n] LDS tile by COLUMNS, which is exactly an
// MFMA operand fragment with 8 consecutive m per lane — so both operands are staged row-major and
// read transposed from LDS (mfma_tile.h, the same images the flash-attention kernels use). No
// transpose pass exists anywhere.
//
// Tile: 256 (n) x 256 (k) output per workgroup, 8 waves as 2 (n) x 4 (k), each wave 128 x 64 =
// 4 x 2 MFMA 32x32x16 accumulators. 32-row m stages of both operands are copied global -> LDS by
// global_load_lds_dwordx4 (no VGPR staging, no ds_write pass): the LDS image is lane-linear, so
// the XOR swizzle that keeps the transposed reads bank-conflict free is applied to the per-lane
// SOURCE address. Four stage buffers form a ring with three stages in flight: a stage waits
// with a counted vmcnt for its own DMA only, then one raw s_barrier publishes it (measured on
// MI355X: with one stage in flight the kernel spent ~35 % of its time waiting for the DMA —
// benchmarks/wgrad_micro.hip). Each buffer is its own __shared__ object so the compiler can
// see that reads of one buffer do not alias the DMA into another and does not drain the queue.
//
// Two launch forms:
//   * smdt_wgrad_accumulate: one GEMM; small outputs are split along m (split-K) to cover the
//     256 CUs and the split partials are added with fp32 atomics (~1.3 TB/s chip-wide, so the
//     split count is chosen against that cost); one split does a plain read-modify-write.
//   * smdt_wgrad_grouped: many independent GEMMs (e.g. several layers' QKV / proj / fc1 / fc2
//     weight gradients queued by the deferred-wgrad path) in ONE launch, every tile over its full
//     m range, deterministic, and the tile count of a whole group fills the machine where a
//     single small GEMM cannot. Only the tiles past the last full round of 256 are split along m
//     with fp32 atomics (see wgrad_grouped_kernel).
// Work items are ordered (problem, n-group, k, n-in-group) and remapped so that the consecutive
// items an XCD runs share A and B strips in that XCD's L2. Partial tiles (N or K not a multiple
// of 256, as the 50304-row LM head) load clamped columns and skip their stores.
#include <cstdlib>

#include "common.h"
#include "launchers.h"
#include "mfma_tile.h"

namespace smdt {
namespace wg {

using namespace mt;
constexpr int BT = 256;              // output tile edge (n and k)
constexpr int BM = 32;               // m rows per stage
using G = Geo<BT>;                   // rows of 512 B, XOR-swizzled 16-byte chunks (row bits 0..3)
constexpr int SB = BM * G::RB;       // bytes per operand stage image (16 KB)
constexpr int kThreads = 512;
constexpr int kWaves = kThreads / 64;
constexpr int kGlds = SB / 1024 / kWaves;  // 1 KB wave-instructions per operand per stage per wave (2)
constexpr int kNBuf = 4;

using lds_void = __attribute__((address_space(3))) void;

// s_waitcnt with vmcnt = n and the other counters left alone (gfx9 encoding).
template <int n>
__device__ __forceinline__ void wait_vm() {
  static_assert(n >= 0 && n < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((n & 15) | ((n >> 4) << 14) | (7 << 4) | (15 << 8));
}

// Copy one 32 x 256 bf16 stage of an operand into its LDS image. Wave instruction i (of 16)
// fills image rows 2i, 2i+1; lane l lands at slot (row 2i + l/32, chunk l%32) and therefore
// loads the global chunk whose swizzled position that is: chunk (l % 32) ^ f(row).
struct Glds {
  int off[kGlds];   // element offsets within the stage (row * ld + clamped column)
  __device__ __forceinline__ void init(int wave, int lane, int ld, int col0, int ncols) {
#pragma unroll
    for (int j = 0; j < kGlds; ++j) {
      const int r = 2 * (wave * kGlds + j) + (lane >> 5);
      const int c = (lane & 31) ^ G::f(r);
      int col = col0 + 8 * c;
      if (col > ncols - 8) col = ncols - 8;  // partial tile: any in-bounds column, never stored
      off[j] = r * ld + col;
    }
  }
  template <class E>
  __device__ __forceinline__ void issue(const E* stage_base, char* img, int wave) const {
#pragma unroll
    for (int j = 0; j < kGlds; ++j)
      __builtin_amdgcn_global_load_lds((const void*)(stage_base + off[j]),
                                       (lds_void*)(img + (wave * kGlds + j) * 1024), 16, 0, 0);
  }
};

// One 256 x 256 output tile over stages [0, nst) of 32 rows starting at A/B row mstart.
// VAR is a diagnostic knob for benchmarks/wgrad_micro.hip only (the library uses VAR = 0):
// bit 0 skips the in-loop DMA, bit 2 the fragment reads. (A v_mfma_f32_16x16x32 form of this
// tile measured +1.7 % on the grouped microbenchmark and neutral-to-slower in the training step,
// profiles/r3_wgrad16/: the kernel is bound by its LDS-DMA operand stream, not by the MFMA clock;
// it was removed.)

// BIAS (the k0 == 0 tiles of a problem with a bias): bias[n0 + r] += sum over this tile's m range
// of A[m, n0 + r] — the bias gradient of the linear whose weight gradient this is, from the A (dY)
// fragments the MFMAs read anyway. All four wk waves of a wn read the same A fragments; wave wk
// sums fragment wk, which it processes first (its accumulators are rotated by wk, so the choice is
// a compile-time index): ~16 VALU per 8 MFMAs on these tiles, on the vector pipe the MFMA-bound
// loop leaves idle, no extra LDS reads (replaces the col_sum_rows +
// col_partials_reduce kernels). Tiles without a bias run the BIAS = false instantiation, i.e. the
// round-3 loop. Earlier forms, measured on the GPT-2 345M step (profiles/r4_wgrad_bias/): a fp32
// VALU sum of the fragment was if-converted by the compiler into sums of all four fragments on
// every tile (35.8 -> 45.0 ms of grouped wgrad); picking fragment wk inside the i loop made it
// branch around an MFMA per fragment (bias tiles ~2.5x slower: 37.0 -> 43.8 ms); the re-read
// fragment times an all-ones B operand (one extra MFMA per 8), or the re-read fragment summed by
// VALU, both cost ~2.7 ms (39.7 / 40.4 ms): the tiles of a launch run in rounds of 256, so a slower
// k = 0 tile in every round stretches every round.
// Sum of the 8 16-bit values of an operand fragment, in fp32.
template <class V>
__device__ __forceinline__ float sum8(V x) {
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) s += (float)x[j];
  return s;
}

template <bool ATOMIC, int VAR, bool BIAS, class E>
__device__ __forceinline__ void tile_gemm(const E* __restrict__ A, const E* __restrict__ B,
                                          float* __restrict__ C, int N, int K, int n0, int k0, int64_t mstart,
                                          int nst, char* L0, char* L1, char* L2, char* L3,
                                          float* __restrict__ bias = nullptr, bool ovw = false) {
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), h = lane >> 5;
  const int wn = wave >> 2, wk = wave & 3;  // wave tile: n rows [128 wn, +128), k cols [64 wk, +64)
  using F = Frag<BT, E>;
  using V = v8_t<E>;
  int oa[4][2], ob[2][2];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    // accumulator i holds the wave's A fragment (i + wk) & 3: every wave meets ITS bias fragment
    // (wk) first, at compile-time index 0 (the output rows follow in the epilogue)
    oa[i][0] = F::tr_off(lane, 4 * wn + ((i + wk) & 3), 0);
    oa[i][1] = F::tr_off(lane, 4 * wn + ((i + wk) & 3), 1);
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    ob[j][0] = F::tr_off(lane, 2 * wk + j, 0);
    ob[j][1] = F::tr_off(lane, 2 * wk + j, 1);
  }
  f32x16 acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = zero16();
  // BIAS: column sums of A over the fragment i == wk, replicated in every column of accb. That
  // fragment is read a second time by its own offsets (wk is only known at run time; selecting it
  // from the four fragments of the i loop made the compiler branch around an MFMA per fragment)
  float cs = 0.f;  // fp32 sum of this lane's 8 rows of column (lane & 31) of fragment wk

  Glds ga, gb;
  ga.init(wave, lane, N, n0, N);
  gb.init(wave, lane, K, k0, K);
  const E* Ab = A + mstart * N;
  const E* Bb = B + mstart * K;
  const int64_t sa = (int64_t)BM * N, sbk = (int64_t)BM * K;

  auto issue = [&](int s, char* img) {
    ga.issue(Ab + s * sa, img, wave);
    gb.issue(Bb + s * sbk, img + SB, wave);
  };
  // Prologue: stages 0 .. kNBuf-2 in flight, wait for stage 0. Every stage issues exactly one
  // DMA (past the end it re-reads the last stage into a buffer nobody reads again), so the
  // counted waits below are uniform and the compiler's own wait insertion stays out of the loop.
  issue(0, L0);
  issue(min(1, nst - 1), L1);
  issue(min(2, nst - 1), L2);
  wait_vm<2 * 2 * kGlds>();
  __builtin_amdgcn_s_barrier();

  // Stage s: prefetch stage s+kNBuf-1 into `pre` (the buffer stage s-1 read, released by the
  // barrier that ended it), MFMA over `cur`, retire stage s+1's DMA, barrier.
  auto stage = [&](int s, const char* cur, char* pre) {
    if (!(VAR & 1)) issue(min(s + kNBuf - 1, nst - 1), pre);
    const char* at = cur;
    const char* bt = cur + SB;
#pragma unroll
    for (int ks = 0; ks < BM / 16; ++ks) {
      V b0, b1;
      if constexpr (VAR & 4) {
        const f32x4 t4 = {acc[0][0][4 * ks], acc[0][1][4 * ks], acc[1][0][4 * ks], acc[1][1][4 * ks]};
        b0 = __builtin_bit_cast(V, t4);
        b1 = b0;
      } else {
        b0 = F::trf_at(bt, 0, ks, ob[0][0], ob[0][1]);
        b1 = F::trf_at(bt, 0, ks, ob[1][0], ob[1][1]);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        V a;
        if constexpr (VAR & 4) a = b1;
        else a = F::trf_at(at, 0, ks, oa[i][0], oa[i][1]);
        acc[i][0] = mfma(a, b0, acc[i][0]);
        acc[i][1] = mfma(a, b1, acc[i][1]);
        if constexpr (BIAS) {
          if (i == 0) cs += sum8(a);   // fragment wk (see oa)
        }
      }
    }
    // Stages s+2 .. s+kNBuf-1 stay in flight; stage s+1 must have landed.
    wait_vm<(kNBuf - 2) * 2 * kGlds>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  };
  int s = 0;
  for (; s + kNBuf <= nst; s += kNBuf) {
    stage(s, L0, L3);
    stage(s + 1, L1, L0);
    stage(s + 2, L2, L1);
    stage(s + 3, L3, L2);
  }
  if (s < nst) stage(s, L0, L3);
  if (s + 1 < nst) stage(s + 1, L1, L0);
  if (s + 2 < nst) stage(s + 2, L2, L1);
  wait_vm<0>();  // drain the trailing re-reads before the workgroup's LDS is released

  if constexpr (BIAS) {
    // lanes l and l ^ 32 summed the two 8-row halves of each 16-row k-step of one column
    cs = __shfl_xor(cs, 32, 64) + cs;
    const int n = n0 + 128 * wn + 32 * wk + (lane & 31);
    if (h == 0 && n < N) {
      if constexpr (ATOMIC) unsafeAtomicAdd(bias + n, cs);
      else bias[n] += cs;
    }
  }

  // Epilogue: register r of acc[i][j] is C[n0 + 128 wn + 32 i + acc_row(r, h)][k0 + 64 wk + 32 j + lane&31];
  // the 32 lanes of a half write 32 consecutive fp32 (128 B) per register. Full 32-row blocks
  // issue all 16 loads before the adds (one round trip per block, not per element).
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int k = k0 + 64 * wk + 32 * j + (lane & 31);
    const bool kok = k < K;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int nb = n0 + 128 * wn + 32 * ((i + wk) & 3);
      float* cp = C + (int64_t)nb * K + k;
      if (nb + 32 <= N && kok) {
        if constexpr (ATOMIC) {
#pragma unroll
          for (int r2 = 0; r2 < 16; ++r2) unsafeAtomicAdd(cp + (int64_t)acc_row(r2, h) * K, acc[i][j][r2]);
        } else if (ovw) {   // first gradient of the step into an unzeroed buffer: store only
#pragma unroll
          for (int r2 = 0; r2 < 16; ++r2) cp[(int64_t)acc_row(r2, h) * K] = acc[i][j][r2];
        } else {
          float old[16];
#pragma unroll
          for (int r2 = 0; r2 < 16; ++r2) old[r2] = cp[(int64_t)acc_row(r2, h) * K];
#pragma unroll
          for (int r2 = 0; r2 < 16; ++r2) cp[(int64_t)acc_row(r2, h) * K] = old[r2] + acc[i][j][r2];
        }
      } else if (kok) {
        for (int r2 = 0; r2 < 16; ++r2) {
          const int rr = acc_row(r2, h);
          if (nb + rr >= N) continue;
          float* p = cp + (int64_t)rr * K;
          if constexpr (ATOMIC)
            unsafeAtomicAdd(p, acc[i][j][r2]);
          else
            *p = ovw ? acc[i][j][r2] : *p + acc[i][j][r2];
        }
      }
    }
  }
}

// XCD-aware bijective remap: hardware dispatches block b to XCD b % 8; give each XCD a
// contiguous range of work items.
__device__ __forceinline__ int xcd_remap(int orig, int nblocks) {
  const int xcd = orig & 7, q = nblocks >> 3, rem = nblocks & 7;
  return (xcd < rem ? xcd * (q + 1) : rem * (q + 1) + (xcd - rem) * q) + (orig >> 3);
}

// Tile t of an ntn x ntk grid in groups of gn n-tiles x all k-tiles, n fastest inside a group.
__device__ __forceinline__ void tile_coords(int t, int ntn, int ntk, int gn, int& tn, int& tk) {
  const int grp = t / (gn * ntk);
  const int gn_eff = min(gn, ntn - grp * gn);
  const int tg = t - grp * gn * ntk;
  tn = grp * gn + tg % gn_eff;
  tk = tg / gn_eff;
}

#define WG_LDS                                                    \
  __shared__ __attribute__((aligned(1024))) char L0[2 * SB];      \
  __shared__ __attribute__((aligned(1024))) char L1[2 * SB];      \
  __shared__ __attribute__((aligned(1024))) char L2[2 * SB];      \
  __shared__ __attribute__((aligned(1024))) char L3[2 * SB];

template <bool ATOMIC, int VAR = 0, class E = bf16>
__global__ __launch_bounds__(kThreads, 1) void wgrad_kernel(const E* __restrict__ A, const E* __restrict__ B,
                                                          float* __restrict__ C, int M, int N, int K, int ntn,
                                                          int ntk, int gn, int m_per_split, int nblocks) {
  WG_LDS
  const int w = xcd_remap(blockIdx.x, nblocks);
  const int tiles = ntn * ntk;
  const int split = w / tiles;
  int tn, tk;
  tile_coords(w - split * tiles, ntn, ntk, gn, tn, tk);
  const int mstart = split * m_per_split;
  const int nst = (min(M, mstart + m_per_split) - mstart) / BM;
  tile_gemm<ATOMIC, VAR, false, E>(A, B, C, N, K, tn * BT, tk * BT, mstart, nst, L0, L1, L2, L3);
}

struct Problem {
  const void* A;
  const void* B;
  float* C;
  float* bias;     // column sums of A (bias gradient) or null
  int M, N, K, ntn, ntk, gn, tile0;
  int ovw;         // C holds no data yet: the epilogue stores instead of read-add-store
};
constexpr int kMaxGroup = 32;
struct Group {
  Problem p[kMaxGroup];
  int nprob;
  int nfull;    // blocks 0 .. nfull-1: whole tiles (a multiple of 256 when a tail is split)
  int splits;   // the tail tiles nfull .. : `splits` blocks each, `mps` stages of the m range apiece
  int mps;
};

// The problem table travels in the kernel arguments (< 2 KB), read from the kernarg segment.
//
// Tail split: whole tiles run in rounds of 256 (one workgroup per CU), so a launch of 256 q + r
// tiles costs q + 1 full rounds even when r is small. The GPT-2 345M LM head alone is
// 197 x 4 = 788 tiles (3 rounds + 20), so every step paid a round with 236 CUs idle. The last r
// tiles of the launch are therefore cut along m into ~256 / r pieces that run together in one
// short round and add their partial sums with fp32 atomics (tail tiles only: their sum order is
// not fixed; everything else stays deterministic). The whole tiles keep the XCD-aware order; the
// pieces go round-robin over the XCDs.
template <class E>
__global__ __launch_bounds__(kThreads, 1) void wgrad_grouped_kernel(const Group g) {
  WG_LDS
  const int bid = blockIdx.x;
  int w, piece = -1;
  if (bid < g.nfull) {
    w = xcd_remap(bid, g.nfull);
  } else {
    const int j = bid - g.nfull;
    w = g.nfull + j / g.splits;
    piece = j % g.splits;
  }
  int pi = 0;
  while (pi + 1 < g.nprob && w >= g.p[pi + 1].tile0) ++pi;
  const Problem& P = g.p[pi];
  int tn, tk;
  tile_coords(w - P.tile0, P.ntn, P.ntk, P.gn, tn, tk);
  const int stages = P.M / BM;
  const bool bias_tile = P.bias != nullptr && tk == 0;
  const E* A = (const E*)P.A;
  const E* B = (const E*)P.B;
  if (piece < 0) {
    if (bias_tile)
      tile_gemm<false, 0, true, E>(A, B, P.C, P.N, P.K, tn * BT, 0, 0, stages, L0, L1, L2, L3, P.bias, P.ovw != 0);
    else
      tile_gemm<false, 0, false, E>(A, B, P.C, P.N, P.K, tn * BT, tk * BT, 0, stages, L0, L1, L2, L3, nullptr,
                                    P.ovw != 0);
  } else {
    const int s0 = piece * g.mps;
    const int nst = min(stages, s0 + g.mps) - s0;
    if (nst <= 0) return;  // a smaller-M problem in the tail: nothing left for this piece (whole block exits)
    if (bias_tile)
      tile_gemm<true, 0, true, E>(A, B, P.C, P.N, P.K, tn * BT, 0, (int64_t)s0 * BM, nst, L0, L1, L2, L3, P.bias);
    else
      tile_gemm<true, 0, false, E>(A, B, P.C, P.N, P.K, tn * BT, tk * BT, (int64_t)s0 * BM, nst, L0, L1, L2, L3);
  }
}

inline int group_width(int ntk) { return ntk <= 4 ? 8 : 4; }

}  // namespace wg
}  // namespace smdt

using namespace smdt;

extern "C" int smdt_wgrad_supported(int64_t M, int64_t N, int64_t K) {
  return M > 0 && M % wg::BM == 0 && N >= 8 && K >= 8 && N % 8 == 0 && K % 8 == 0 && M < (1ll << 31) &&
         N * K < (1ll << 31) && (int64_t)wg::BM * (N > K ? N : K) < (1ll << 31);
}

extern "C" hipError_t smdt_wgrad_accumulate(const void* dy, const void* x, float* main_grad, int64_t M,
                                            int64_t N, int64_t K, int max_splits, hipStream_t st) {
  return smdt_wgrad_accumulate_t(1, dy, x, main_grad, M, N, K, max_splits, st);
}

extern "C" hipError_t smdt_wgrad_accumulate_t(int dtype, const void* dy, const void* x, float* main_grad, int64_t M,
                                              int64_t N, int64_t K, int max_splits, hipStream_t st) {
  if (dtype != 1 && dtype != 2) return hipErrorInvalidValue;
  if (!smdt_wgrad_supported(M, N, K)) return hipErrorInvalidValue;
  const int ntn = (int)((N + wg::BT - 1) / wg::BT), ntk = (int)((K + wg::BT - 1) / wg::BT);
  const int tiles = ntn * ntk;
  const int64_t stages = M / wg::BM;
  // Split count: modelled time = rounds of 256 blocks x (stages per split + the atomic epilogue,
  // which costs about as much as 48 stages of 32 rows when every CU adds a 256 KB partial).
  int splits = 1;
  if (max_splits != 1) {
    const int cap = max_splits > 0 ? max_splits : 16;
    double best_t = 1e30;
    for (int s = 1; s <= cap; ++s) {
      if (s > 1 && stages / s < 8) break;
      const int64_t blocks = (int64_t)tiles * s;
      const int64_t rounds = (blocks + 255) / 256;
      const double per = (double)((stages + s - 1) / s) +
                         (s > 1 ? 48.0 * (double)(blocks < 256 ? blocks : 256) / 256.0 : 0.0);
      const double t = rounds * per;
      if (t < best_t * 0.97) {
        best_t = t;
        splits = s;
      }
    }
  }
  const int m_per_split = (int)(((stages + splits - 1) / splits) * wg::BM);
  splits = (int)((M + m_per_split - 1) / m_per_split);
  const int nblocks = tiles * splits;
  const int gn = wg::group_width(ntk);
#define SMDT_WG(AT, ET)                                                                                      \
  hipLaunchKernelGGL((wg::wgrad_kernel<AT, 0, ET>), dim3(nblocks), dim3(wg::kThreads), 0, st, (const ET*)dy, \
                     (const ET*)x, main_grad, (int)M, (int)N, (int)K, ntn, ntk, gn, m_per_split, nblocks)
  if (dtype == 2) {
    if (splits > 1) SMDT_WG(true, f16); else SMDT_WG(false, f16);
  } else {
    if (splits > 1) SMDT_WG(true, bf16); else SMDT_WG(false, bf16);
  }
#undef SMDT_WG
  return hipGetLastError();
}

static bool wg_tail_split_enabled() {
  static const int on = [] {
    const char* v = getenv("SMDT_WGRAD_TAIL_SPLIT");
    return (v && v[0] == '0') ? 0 : 1;
  }();
  return on != 0;
}

// Grouped form: one launch per 32 problems, the table passed by value.
extern "C" hipError_t smdt_wgrad_grouped(const SmdtWgradProblem* probs, int n, hipStream_t st) {
  return smdt_wgrad_grouped_t(1, probs, n, st);
}

extern "C" hipError_t smdt_wgrad_grouped_t(int dtype, const SmdtWgradProblem* probs, int n, hipStream_t st) {
  return smdt_wgrad_grouped_cus(dtype, probs, n, 0, st);
}

// `cus`: the CUs this launch can use at once (0 = 256). A launch beside a transfer that holds CUs
// (a filler in a TP exchange wait, parallel/tensor_parallel.DeferredWgrad.fill_one) sizes its
// rounds and its tail split to what is left, so no tail piece waits for the transfer to end.
extern "C" hipError_t smdt_wgrad_grouped_cus(int dtype, const SmdtWgradProblem* probs, int n, int cus,
                                             hipStream_t st) {
  if (dtype != 1 && dtype != 2) return hipErrorInvalidValue;
  const int R = (cus > 0 && cus < 256) ? cus : 256;
  for (int i = 0; i < n; ++i)
    if (!smdt_wgrad_supported(probs[i].M, probs[i].N, probs[i].K)) return hipErrorInvalidValue;
  for (int base = 0; base < n; base += wg::kMaxGroup) {
    wg::Group g;
    const int cnt = n - base < wg::kMaxGroup ? n - base : wg::kMaxGroup;
    int tiles = 0;
    for (int i = 0; i < cnt; ++i) {
      const SmdtWgradProblem& q = probs[base + i];
      wg::Problem& p = g.p[i];
      p.A = q.dy;
      p.B = q.x;
      p.C = q.main_grad;
      p.bias = q.bias_grad;
      p.M = (int)q.M;
      p.N = (int)q.N;
      p.K = (int)q.K;
      p.ntn = (int)((q.N + wg::BT - 1) / wg::BT);
      p.ntk = (int)((q.K + wg::BT - 1) / wg::BT);
      p.gn = wg::group_width(p.ntk);
      p.tile0 = tiles;
      p.ovw = q.overwrite ? 1 : 0;
      tiles += p.ntn * p.ntk;
    }
    for (int i = cnt; i < wg::kMaxGroup; ++i) g.p[i] = g.p[cnt - 1];
    g.nprob = cnt;
    // Tail split (see wgrad_grouped_kernel): r = tiles mod 256 tail tiles, ~256 / r pieces each
    // of at least 8 stages; off with SMDT_WGRAD_TAIL_SPLIT=0.
    const int r = tiles % R;
    int splits = 1, mps = 0;
    if (r > 0 && wg_tail_split_enabled()) {
      int max_stages = 0;
      for (int i = 0; i < cnt; ++i) max_stages = max_stages > g.p[i].M / wg::BM ? max_stages : g.p[i].M / wg::BM;
      splits = R / r;
      if (splits > 16) splits = 16;
      if (splits > max_stages / 8) splits = max_stages / 8;
      if (splits > 1) {
        mps = (max_stages + splits - 1) / splits;
        splits = (max_stages + mps - 1) / mps;
      }
    }
    if (splits <= 1) {
      g.nfull = tiles;
      g.splits = 1;
      g.mps = 0;
    } else {
      g.nfull = tiles - r;
      g.splits = splits;
      g.mps = mps;
      // the split tail adds partial sums with atomics: an overwrite problem with tail tiles is
      // zeroed first and accumulates like the rest
      for (int i = 0; i < cnt; ++i) {
        wg::Problem& p = g.p[i];
        if (p.ovw && p.tile0 + p.ntn * p.ntk > g.nfull) {
          hipError_t e = hipMemsetAsync(p.C, 0, (size_t)p.N * (size_t)p.K * sizeof(float), st);
          if (e != hipSuccess) return e;
          p.ovw = 0;
        }
      }
    }
    const int nblocks = g.nfull + (tiles - g.nfull) * g.splits;
    if (dtype == 2)
      hipLaunchKernelGGL((wg::wgrad_grouped_kernel<f16>), dim3(nblocks), dim3(wg::kThreads), 0, st, g);
    else
      hipLaunchKernelGGL((wg::wgrad_grouped_kernel<bf16>), dim3(nblocks), dim3(wg::kThreads), 0, st, g);
  }
  return hipGetLastError();
}
