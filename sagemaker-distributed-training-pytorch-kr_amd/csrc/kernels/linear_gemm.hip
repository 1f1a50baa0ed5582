// Linear-layer forward GEMM with fused epilogues on gfx950 MFMA:
//
//     Y[m, n] = sum_k X[m, k] W[n, k]            (EPI 0)
//     Y[m, n] = sum_k X[m, k] W[n, k] + b[n]     (EPI 1)
//     H = X W^T + b,  Y = GeLU_tanh(H)           (EPI 2: the MLP's fc1 + bias-GeLU, both stored)
//
// X [M, K] and W [N, K] are row-major with the reduction index k CONTIGUOUS in both (the "NT"
// layout of a torch.nn.Linear forward). This replaces Megatron's separate bias-GeLU fusion pass
// after the fc1 GEMM (--no-bias-gelu-fusion, /root/reference/3_training_megatron-lm/
// megatron/arguments.py:819-821): the activation is applied to the fp32 accumulator before the one
// rounding to bf16, and the pre-activation H (needed by the backward's GeLU derivative) is written
// by the same epilogue, so the [tokens, 4h] intermediate makes one trip to HBM instead of three.
//
// Structure (shares mfma_tile.h with the flash-attention and weight-gradient kernels):
//   * 256 x 256 output tile per workgroup, 8 waves as 2 (m) x 4 (n), each wave 128 m x 64 n =
//     8 x 4 accumulators of v_mfma_f32_16x16x32 (bf16 or fp16 operands), one MFMA k-step per stage;
//   * k is staged 32 at a time: a stage of each operand is 256 rows x 64 B, copied global -> LDS by
//     global_load_lds_dwordx4 (1 KB = 16 rows per wave-instruction, no VGPR staging, no ds_write
//     pass) into an XOR-swizzled image (swizzle applied to the per-lane SOURCE address),
//     read back by rows with ds_read_b128, bank-conflict free;
//   * a ring of four stage buffers, three stages in flight: one counted vmcnt + one barrier per
//     stage; the grid is persistent (one workgroup per CU) and the stage stream runs on across a
//     block's tiles, so a tile's epilogue overlaps the DMA of the next tile's first stages;
//   * the "swapped" product D = W . X^T puts the token index m on the MFMA lane and 4 consecutive
//     output features n in registers: the epilogue applies the per-feature bias / GeLU straight
//     from registers and stages each 32-row slab through LDS so every store is a coalesced 16-byte
//     piece of a 128-byte row segment;
//   * tiles are ordered in groups of 8 m-tiles x all n-tiles and remapped so that each XCD runs a
//     contiguous range (the W strip and 8 X strips stay in that XCD's L2).
// Partial tiles (M or N not a multiple of 256, e.g. the 50304-row LM head) load clamped rows and
// skip their stores. Requirements (host-checked): K % 128 == 0, N % 8 == 0, 16-byte aligned rows.
#include <stdlib.h>

#include "activations.h"
#include "common.h"
#include "launchers.h"
#include "mfma_tile.h"

namespace smdt {
namespace lg {

using namespace mt;
constexpr int BT = 256;                  // output tile edge (m and n)
constexpr int BK = 32;                   // k per stage
constexpr int RB = BK * 2;               // bytes per staged row (64)
constexpr int SB = BT * RB;              // bytes per operand stage image (16 KB)
constexpr int kRowsPerInst = 1024 / RB;            // 16 rows per 1-KB wave-instruction
constexpr int kNBuf = 4;                           // stage ring: 3 stages in flight
constexpr int kGroupM = 8;

// Wave layout of the 256 x 256 tile for linear_fwd_kernel: NW = 8 waves as 2 (m) x 4 (n), 128 x 64
// each (12 fragment reads per 32 MFMAs). The 4-wave layout (2 x 2 waves of 128 x 128, 16 reads per
// 64 MFMAs) is linear_fwd_p4_kernel below, software-pipelined because one wave per SIMD has no
// sibling to hide its LDS latency.
template <int NW>
struct Cfg {
  static constexpr int kThreads = 64 * NW;
  static constexpr int WN = NW == 8 ? 64 : 128;          // features per wave
  static constexpr int NI = WN / 16;                      // 16-feature blocks per wave
  static constexpr int kInst = SB / 1024 / NW;            // DMA wave-instructions per operand per stage
  static constexpr int kPer = 2 * kInst;
  static constexpr int ERB = WN * 2;                      // bytes per epilogue LDS row
  static constexpr int ECH = ERB / 16;                    // 16-byte chunks per epilogue row
  static constexpr int ERI = 64 / ECH;                    // epilogue rows per wave-instruction
  __device__ static __forceinline__ int wm(int wave) { return NW == 8 ? wave >> 2 : wave >> 1; }
  __device__ static __forceinline__ int wn(int wave) { return NW == 8 ? wave & 3 : wave & 1; }
};

// 64-byte rows of 4 16-byte chunks; chunk c of row r sits at slot c ^ ((r >> 2) & 3). The 16 lanes
// of a ds_read_b128 quarter-wave read rows r0 .. r0 + 15 at one chunk: (r & 3, (r >> 2) & 3) covers
// all 16 combinations, so the 16 x 16 bytes land in 16 distinct bank groups — conflict free.
__device__ __forceinline__ int swz(int r) { return (r >> 2) & 3; }
__device__ __forceinline__ int lds_off(int r, int c) { return r * RB + 16 * (c ^ swz(r)); }

using lds_void = __attribute__((address_space(3))) void;

__device__ __forceinline__ f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x4 mfma16(f16x8 a, f16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

template <int n>
__device__ __forceinline__ void wait_vm() {
  static_assert(n >= 0 && n < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((n & 15) | ((n >> 4) << 14) | (7 << 4) | (15 << 8));
}

// One operand's 256-row x 32-k stage: wave-instruction I fills image rows 16 I .. 16 I + 15; lane l
// lands at (row 16 I + l / 4, slot l % 4) and loads the global chunk whose swizzled slot that is.
// Offsets are relative to the tile's first row; rows past the end are clamped (never stored).
template <int kInst>
struct Glds {
  int rel[kInst];  // row * ld + 8 * chunk of this lane's piece, relative to the tile origin
  __device__ __forceinline__ void init(int wave, int lane, int ld, int row0, int nrows) {
#pragma unroll
    for (int j = 0; j < kInst; ++j) {
      const int r = (wave * kInst + j) * kRowsPerInst + lane / 4;
      const int c = (lane % 4) ^ swz(r);
      int row = row0 + r;
      if (row > nrows - 1) row = nrows - 1;
      rel[j] = (row - row0) * ld + 8 * c;
    }
  }
  template <class E>
  __device__ __forceinline__ void issue(const E* base, char* img, int wave) const {
#pragma unroll
    for (int j = 0; j < kInst; ++j)
      __builtin_amdgcn_global_load_lds((const void*)(base + rel[j]), (lds_void*)(img + (wave * kInst + j) * 1024), 16,
                                       0, 0);
  }
};

// Persistent-grid tile order: round r of the grid gives XCD x (blocks b with b % 8 == x) the 32
// consecutive tiles r * G + 32 x .., and tiles are numbered in groups of kGroupM m-tiles x all
// n-tiles (m fastest), so an XCD's concurrent tiles share 8 X strips and a few W strips in its L2.
__device__ __forceinline__ void tile_of(int t, int ntm, int ntn, int& tm, int& tn) {
  const int grp = t / (kGroupM * ntn);
  const int gm = min(kGroupM, ntm - grp * kGroupM);
  const int tg = t - grp * kGroupM * ntn;
  tm = grp * kGroupM + tg % gm;
  tn = tg / gm;
}

template <int EPI, class E, int NW>
__global__ __launch_bounds__(64 * NW, 1) void linear_fwd_kernel(const E* __restrict__ X, const E* __restrict__ W,
                                                                 const E* __restrict__ bias, E* __restrict__ Y,
                                                                 E* __restrict__ H, int M, int N, int K, int ldx,
                                                                 int ldw, int ldy, int ntm, int ntn) {
  __shared__ __attribute__((aligned(1024))) char L0[2 * SB];
  __shared__ __attribute__((aligned(1024))) char L1[2 * SB];
  __shared__ __attribute__((aligned(1024))) char L2[2 * SB];
  __shared__ __attribute__((aligned(1024))) char L3[2 * SB];
  const int ntiles = ntm * ntn;
  const int G = gridDim.x;
  const int b = blockIdx.x;
  // logical tile of this block's i-th round (XCD-contiguous ranges, see tile_of)
  const int xcd = b & 7, slot = b >> 3, per_xcd = G >> 3;
  auto logical = [&](int i) { return i * G + xcd * per_xcd + slot; };
  int my_tiles = 0;
  while (logical(my_tiles) < ntiles) ++my_tiles;

  using C = Cfg<NW>;
  constexpr int NI = C::NI, WN = C::WN, kPer = C::kPer;
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = C::wm(wave), wn = C::wn(wave);  // wave tile: m [128 wm, +128), n [WN wn, +WN)
  using V = v8_t<E>;
  // v_mfma_f32_16x16x32: lane l holds rows (l & 15) of a 16-row operand block at k = 8 (l >> 4) .. +8,
  // i.e. 16-byte chunk (l >> 4) of the 64-byte staged row; the 4 result registers are rows
  // 4 (l >> 4) .. +4 (features), column l & 15 (token). 16x16x32 rather than 32x32x16: the chip
  // holds a higher clock on it (MI355X_MICROARCH.md, DVFS give-back item 7), same cycles per FLOP.
  const int l15 = lane & 15, lq = lane >> 4;
  const int rdo = lds_off(l15, lq);

  const int nst = K / BK;  // a multiple of kNBuf: every tile starts at ring position 0
  // DMA cursor over this block's stage stream: tile di, stage ds (past the end: the last stage
  // again, re-read into a buffer nobody reads any more, so every step issues exactly one stage)
  Glds<C::kInst> gx, gw;
  int di = 0, ds = 0;
  const E* Xb = X;
  const E* Wb = W;
  auto set_tile = [&](int i) {
    int tm, tn;
    tile_of(logical(i), ntm, ntn, tm, tn);
    gx.init(wave, lane, ldx, tm * BT, M);
    gw.init(wave, lane, ldw, tn * BT, N);
    Xb = X + (int64_t)tm * BT * ldx;
    Wb = W + (int64_t)tn * BT * ldw;
  };
  auto issue_next = [&](char* img) {
    gx.issue(Xb + ds * BK, img, wave);
    gw.issue(Wb + ds * BK, img + SB, wave);
    if (++ds == nst) {
      if (di + 1 < my_tiles) {
        ++di;
        ds = 0;
        set_tile(di);
      } else {
        ds = nst - 1;
      }
    }
  };

  f32x4 acc[NI][8];  // [16-feature block ni][16-token block mi] of the wave's WN x 128 tile
#pragma unroll
  for (int j = 0; j < NI; ++j)
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};

  // Epilogue of tile i, staged through this wave's 4 KB of L3 (free here: the tile's last step read
  // it, the next tile's first step refills it after the closing barrier). Per 32-token slab the
  // wave writes its 32 x 64 block row-major (16-byte chunk c of row m at slot c ^ (m & 7)), reads
  // it back 16 B per lane and stores whole 128-byte row segments: 4 coalesced dwordx4 stores per
  // slab instead of 8 dwordx2 stores that touch 64 rows each (the store-issue-bound tail,
  // MI355X_MICROARCH.md "attention epilogue store tail").
  char* const wreg = L3 + wave * (32 * C::ERB);
  auto slab_out = [&](E* __restrict__ out, int mb, int nb) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int q = 0; q < 32 / C::ERI; ++q) {
      const int row = C::ERI * q + lane / C::ECH, c = lane % C::ECH;
      const v8_t<E> v = *reinterpret_cast<const v8_t<E>*>(wreg + row * C::ERB + 16 * (c ^ (row % C::ECH)));
      const int m = mb + row, n = nb + 8 * c;
      if (m < M && n < N) *reinterpret_cast<v8_t<E>*>(out + (int64_t)m * ldy + n) = v;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  };
  auto epilogue = [&](int i) {
    int tm, tn;
    tile_of(logical(i), ntm, ntn, tm, tn);
    const int m0 = tm * BT, n0 = tn * BT;
    // register r of acc[ni][mi] = D[n = 64 wn + 16 ni + 4 lq + r][m = 128 wm + 16 mi + l15]
    float bv[NI][4];
#pragma unroll
    for (int ni = 0; ni < NI; ++ni) {
      const int n = n0 + WN * wn + 16 * ni + 4 * lq;
#pragma unroll
      for (int e = 0; e < 4; ++e) bv[ni][e] = 0.f;
      if constexpr (EPI >= 1) {
        if (n < N) {
          const v4_t<E> b4 = *reinterpret_cast<const v4_t<E>*>(bias + n);
#pragma unroll
          for (int e = 0; e < 4; ++e) bv[ni][e] = (float)b4[e];
        }
      }
    }
#pragma unroll
    for (int sl = 0; sl < 4; ++sl) {  // 32-token slabs: token blocks mi = 2 sl, 2 sl + 1
      const int mb = m0 + 128 * wm + 32 * sl, nb = n0 + WN * wn;
#pragma unroll
      for (int pass = 0; pass < (EPI == 2 ? 2 : 1); ++pass) {  // EPI 2: pre-activation, then GeLU
#pragma unroll
        for (int half = 0; half < 2; ++half) {
          const int row = 16 * half + l15;
#pragma unroll
          for (int ni = 0; ni < NI; ++ni) {
            v4_t<E> v;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const float x = acc[ni][2 * sl + half][e] + bv[ni][e];
              v[e] = (E)(EPI == 2 && pass == 1 ? gelu_tanh(x) : x);
            }
            const int c = 2 * ni + (lq >> 1);  // 16-byte chunk of the LDS row
            *reinterpret_cast<v4_t<E>*>(wreg + row * C::ERB + 16 * (c ^ (row % C::ECH)) + 8 * (lq & 1)) = v;
          }
        }
        slab_out(EPI == 2 && pass == 0 ? H : Y, mb, nb);
      }
    }
#pragma unroll
    for (int j = 0; j < NI; ++j)
#pragma unroll
      for (int ii = 0; ii < 8; ++ii) acc[j][ii] = f32x4{0.f, 0.f, 0.f, 0.f};
    __builtin_amdgcn_s_barrier();  // every wave is done with L3 before the next step's DMA into it
  };
  // global stores one epilogue leaves in flight per wave (they count in vmcnt)
  constexpr int kEpiStores = 4 * (32 / C::ERI) * (EPI == 2 ? 2 : 1);
  constexpr int kRelaxedWait = (kNBuf - 2) * kPer + kEpiStores < 63 ? (kNBuf - 2) * kPer + kEpiStores : 63;

  if (my_tiles == 0) return;
  set_tile(0);
  // Prologue: stages 0 .. 2 in flight, wait for stage 0.
  issue_next(L0);
  issue_next(L1);
  issue_next(L2);
  wait_vm<2 * kPer>();
  __builtin_amdgcn_s_barrier();

  // One step: prefetch the stage 3 ahead into `pre` (the buffer the previous step read, released
  // by the barrier that ended it), MFMA over `cur`, retire the next stage's DMA, barrier.
  // kRelaxed: the first step after an epilogue, whose stores sit between the DMA it waits for and
  // the newest one.
  auto step = [&](const char* cur, char* pre, auto relaxed) {
    issue_next(pre);
    __builtin_amdgcn_sched_barrier(0);  // keep the DMA at the head of the step (the scheduler sinks it)
    const char* xt = cur;
    const char* wt = cur + SB;
    // NI feature fragments + 8 token fragments feed 8 NI MFMAs
    V wf[NI];
#pragma unroll
    for (int ni = 0; ni < NI; ++ni) wf[ni] = *reinterpret_cast<const V*>(wt + (WN * wn + 16 * ni) * RB + rdo);
#pragma unroll
    for (int mi = 0; mi < 8; ++mi) {
      const V xf = *reinterpret_cast<const V*>(xt + (128 * wm + 16 * mi) * RB + rdo);
#pragma unroll
      for (int ni = 0; ni < NI; ++ni) acc[ni][mi] = mfma16(wf[ni], xf, acc[ni][mi]);  // D[n][m]
    }
    if constexpr (decltype(relaxed)::value)
      wait_vm<kRelaxedWait>();
    else
      wait_vm<(kNBuf - 2) * kPer>();  // the next stage landed (two more may still be in flight)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  };
  using Strict = std::integral_constant<bool, false>;
  using Relaxed = std::integral_constant<bool, true>;
  for (int i = 0; i < my_tiles; ++i) {
    if (i == 0) step(L0, L3, Strict{});
    else step(L0, L3, Relaxed{});
    step(L1, L0, Strict{});
    step(L2, L1, Strict{});
    step(L3, L2, Strict{});
    for (int st = kNBuf; st < nst; st += kNBuf) {
      step(L0, L3, Strict{});
      step(L1, L0, Strict{});
      step(L2, L1, Strict{});
      step(L3, L2, Strict{});
    }
    // the next tile's first three stages are in flight while this tile's results are stored
    epilogue(i);
  }
  wait_vm<0>();  // drain the trailing re-reads (and the last stores) before the LDS is released
}


// 4-wave software-pipelined variant: each wave owns 128 m x 128 n (8 x 8 accumulators of
// v_mfma_f32_16x16x32, 256 AGPRs; half the LDS fragment bytes per MFMA of the 8-wave layout) and,
// with one wave per SIMD, hides its own LDS latency: the fragments of stage s + 1 are read while
// the second half of stage s's MFMAs runs. One barrier per stage sits in the MIDDLE of the stage:
// it publishes stage s + 1's DMA to every wave and certifies that every wave has consumed stage s's
// fragments, so the DMA of stage s + 4 is issued into stage s's buffer right after it (four
// buffers, three stages in flight while one is read). The epilogue stages through its own 16 KB
// (the ring is busy with the next tile's stages) in 16-row slabs.
template <int EPI, class E>
__global__ __launch_bounds__(256, 1) void linear_fwd_p4_kernel(const E* __restrict__ X, const E* __restrict__ W,
                                                               const E* __restrict__ bias, E* __restrict__ Y,
                                                               E* __restrict__ H, int M, int N, int K, int ldx,
                                                               int ldw, int ldy, int ntm, int ntn) {
  __shared__ __attribute__((aligned(1024))) char L0[2 * SB];
  __shared__ __attribute__((aligned(1024))) char L1[2 * SB];
  __shared__ __attribute__((aligned(1024))) char L2[2 * SB];
  __shared__ __attribute__((aligned(1024))) char L3[2 * SB];
  constexpr int ERB = 256;  // epilogue LDS row: 128 features x 2 B
  __shared__ __attribute__((aligned(1024))) char LE[4 * 16 * ERB];
  constexpr int kInst = SB / 1024 / 4;  // DMA wave-instructions per operand per stage (4)
  constexpr int kPer = 2 * kInst;
  const int ntiles = ntm * ntn;
  const int G = gridDim.x;
  const int b = blockIdx.x;
  const int xcd = b & 7, slot = b >> 3, per_xcd = G >> 3;
  auto logical = [&](int i) { return i * G + xcd * per_xcd + slot; };
  int my_tiles = 0;
  while (logical(my_tiles) < ntiles) ++my_tiles;
  if (my_tiles == 0) return;

  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave >> 1, wn = wave & 1;  // wave tile: m [128 wm, +128), n [128 wn, +128)
  using V = v8_t<E>;
  const int l15 = lane & 15, lq = lane >> 4;
  const int rdo = lds_off(l15, lq);
  const int nst = K / BK;  // a multiple of 4: every tile starts at ring position 0

  Glds<kInst> gx, gw;
  int di = 0, ds = 0;
  const E* Xb = X;
  const E* Wb = W;
  auto set_tile = [&](int i) {
    int tm, tn;
    tile_of(logical(i), ntm, ntn, tm, tn);
    gx.init(wave, lane, ldx, tm * BT, M);
    gw.init(wave, lane, ldw, tn * BT, N);
    Xb = X + (int64_t)tm * BT * ldx;
    Wb = W + (int64_t)tn * BT * ldw;
  };
  auto issue_next = [&](char* img) {
    gx.issue(Xb + ds * BK, img, wave);
    gw.issue(Wb + ds * BK, img + SB, wave);
    if (++ds == nst) {
      if (di + 1 < my_tiles) {
        ++di;
        ds = 0;
        set_tile(di);
      } else {
        ds = nst - 1;
      }
    }
  };

  f32x4 acc[8][8];  // [16-feature block ni][16-token block mi]
#pragma unroll
  for (int j = 0; j < 8; ++j)
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
  V fa_w[8], fa_x[8], fb_w[8], fb_x[8];  // two fragment sets (stage s, stage s + 1)

  auto load_frags = [&](const char* buf, V (&fw)[8], V (&fx)[8]) {
#pragma unroll
    for (int ni = 0; ni < 8; ++ni) fw[ni] = *reinterpret_cast<const V*>(buf + SB + (128 * wn + 16 * ni) * RB + rdo);
#pragma unroll
    for (int mi = 0; mi < 8; ++mi) fx[mi] = *reinterpret_cast<const V*>(buf + (128 * wm + 16 * mi) * RB + rdo);
  };
  auto half = [&](const V (&fw)[8], const V (&fx)[8], int h) {
#pragma unroll
    for (int mi = 4 * h; mi < 4 * h + 4; ++mi)
#pragma unroll
      for (int ni = 0; ni < 8; ++ni) acc[ni][mi] = mfma16(fw[ni], fx[mi], acc[ni][mi]);  // D[n][m]
  };

  char* const wreg = LE + wave * (16 * ERB);
  auto epilogue = [&](int i) {
    int tm, tn;
    tile_of(logical(i), ntm, ntn, tm, tn);
    const int m0 = tm * BT, n0 = tn * BT;
    float bv[8][4];
#pragma unroll
    for (int ni = 0; ni < 8; ++ni) {
      const int n = n0 + 128 * wn + 16 * ni + 4 * lq;
#pragma unroll
      for (int e = 0; e < 4; ++e) bv[ni][e] = 0.f;
      if constexpr (EPI >= 1) {
        if (n < N) {
          const v4_t<E> b4 = *reinterpret_cast<const v4_t<E>*>(bias + n);
#pragma unroll
          for (int e = 0; e < 4; ++e) bv[ni][e] = (float)b4[e];
        }
      }
    }
#pragma unroll
    for (int mi = 0; mi < 8; ++mi) {  // 16-token slabs
      const int mb = m0 + 128 * wm + 16 * mi, nb = n0 + 128 * wn;
#pragma unroll
      for (int pass = 0; pass < (EPI == 2 ? 2 : 1); ++pass) {
#pragma unroll
        for (int ni = 0; ni < 8; ++ni) {
          v4_t<E> v;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float x = acc[ni][mi][e] + bv[ni][e];
            v[e] = (E)(EPI == 2 && pass == 1 ? gelu_tanh(x) : x);
          }
          const int c = 2 * ni + (lq >> 1);  // 16-byte chunk of the 256-byte LDS row l15
          *reinterpret_cast<v4_t<E>*>(wreg + l15 * ERB + 16 * (c ^ l15) + 8 * (lq & 1)) = v;
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        E* __restrict__ out = EPI == 2 && pass == 0 ? H : Y;
#pragma unroll
        for (int q = 0; q < 4; ++q) {  // 4 rows x 16 chunks per wave-instruction
          const int row = 4 * q + lane / 16, c = lane % 16;
          const V v = *reinterpret_cast<const V*>(wreg + row * ERB + 16 * (c ^ row));
          const int m = mb + row, n = nb + 8 * c;
          if (m < M && n < N) *reinterpret_cast<V*>(out + (int64_t)m * ldy + n) = v;
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
      for (int ii = 0; ii < 8; ++ii) acc[j][ii] = f32x4{0.f, 0.f, 0.f, 0.f};
  };
  constexpr int kEpiStores = 4 * 8 * (EPI == 2 ? 2 : 1);
  constexpr int kRelaxedWait = 2 * kPer + kEpiStores < 63 ? 2 * kPer + kEpiStores : 63;

  set_tile(0);
  issue_next(L0);
  issue_next(L1);
  issue_next(L2);
  issue_next(L3);
  wait_vm<3 * kPer>();
  asm volatile("s_barrier" ::: "memory");
  load_frags(L0, fa_w, fa_x);

  // Step over stage s (fragments in F, buffer cur), next stage's buffer nxt.
  auto step = [&](char* cur, const char* nxt, V (&Fw)[8], V (&Fx)[8], V (&Gw)[8], V (&Gx)[8], auto relaxed) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // F landed
    half(Fw, Fx, 0);
    if constexpr (decltype(relaxed)::value)
      wait_vm<kRelaxedWait>();
    else
      wait_vm<2 * kPer>();  // stage s + 1 landed (s + 2, s + 3 may still be in flight)
    asm volatile("s_barrier" ::: "memory");
    issue_next(cur);  // stage s + 4 into the buffer every wave has finished reading
    load_frags(nxt, Gw, Gx);
    __builtin_amdgcn_sched_barrier(0);
    half(Fw, Fx, 1);
  };
  using Strict = std::integral_constant<bool, false>;
  using Relaxed = std::integral_constant<bool, true>;
  for (int i = 0; i < my_tiles; ++i) {
    if (i == 0) step(L0, L1, fa_w, fa_x, fb_w, fb_x, Strict{});
    else step(L0, L1, fa_w, fa_x, fb_w, fb_x, Relaxed{});
    step(L1, L2, fb_w, fb_x, fa_w, fa_x, Strict{});
    step(L2, L3, fa_w, fa_x, fb_w, fb_x, Strict{});
    step(L3, L0, fb_w, fb_x, fa_w, fa_x, Strict{});
    for (int st = 4; st < nst; st += 4) {
      step(L0, L1, fa_w, fa_x, fb_w, fb_x, Strict{});
      step(L1, L2, fb_w, fb_x, fa_w, fa_x, Strict{});
      step(L2, L3, fa_w, fa_x, fb_w, fb_x, Strict{});
      step(L3, L0, fb_w, fb_x, fa_w, fa_x, Strict{});
    }
    epilogue(i);
  }
  wait_vm<0>();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
}

}  // namespace lg
}  // namespace smdt

using namespace smdt;

extern "C" int smdt_linear_fwd_supported(int64_t M, int64_t N, int64_t K) {
  return M > 0 && N >= 8 && K >= lg::BK * lg::kNBuf && K % (lg::BK * lg::kNBuf) == 0 && N % 8 == 0 && M < (1ll << 31) &&
         (int64_t)lg::BT * (K > N ? K : N) < (1ll << 31) && M * K < (1ll << 31) && N * K < (1ll << 31) &&
         M * N < (1ll << 31);
}

// epi: 0 = plain, 1 = + bias, 2 = + bias -> GeLU(tanh) into y with the pre-activation into h.
// waves: 8 or 4 (wave layouts, see Cfg); 0 = the default (SMDT_LINEAR_WAVES, else 8).
extern "C" hipError_t smdt_linear_fwd(int dtype, int epi, const void* x, const void* w, const void* bias, void* y,
                                      void* h, int64_t M, int64_t N, int64_t K, int64_t ldx, int64_t ldw,
                                      int64_t ldy, int waves, hipStream_t st) {
  static int def_waves = 0;
  if (!def_waves) {
    const char* e = getenv("SMDT_LINEAR_WAVES");
    def_waves = (e && atoi(e) == 4) ? 4 : 8;
  }
  if (waves == 0) waves = def_waves;
  if (waves != 4 && waves != 8) return hipErrorInvalidValue;
  if (dtype != 1 && dtype != 2) return hipErrorInvalidValue;
  if (epi < 0 || epi > 2 || !smdt_linear_fwd_supported(M, N, K)) return hipErrorInvalidValue;
  if ((epi >= 1 && !bias) || (epi == 2 && !h)) return hipErrorInvalidValue;
  if (ldx % 8 || ldw % 8 || ldy % 8 || ldx < K || ldw < K || ldy < N) return hipErrorInvalidValue;
  const int ntm = (int)((M + lg::BT - 1) / lg::BT), ntn = (int)((N + lg::BT - 1) / lg::BT);
  // persistent grid: one workgroup per CU (a multiple of 8 so every XCD gets the same share)
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      cus = 256;
  }
  int nb = ntm * ntn < cus ? ntm * ntn : cus;
  nb = (nb + 7) / 8 * 8;
  const dim3 grid((unsigned)nb);
#define SMDT_LG1(EP, ET, NW)                                                                                       \
  hipLaunchKernelGGL((lg::linear_fwd_kernel<EP, ET, NW>), grid, dim3(64 * NW), 0, st, (const ET*)x, (const ET*)w,  \
                     (const ET*)bias, (ET*)y, (ET*)h, (int)M, (int)N, (int)K, (int)ldx, (int)ldw, (int)ldy, ntm, ntn)
#define SMDT_LG4(EP, ET)                                                                                          \
  hipLaunchKernelGGL((lg::linear_fwd_p4_kernel<EP, ET>), grid, dim3(256), 0, st, (const ET*)x, (const ET*)w,          \
                     (const ET*)bias, (ET*)y, (ET*)h, (int)M, (int)N, (int)K, (int)ldx, (int)ldw, (int)ldy, ntm, ntn)
#define SMDT_LG(EP, ET) \
  do { if (waves == 4) SMDT_LG4(EP, ET); else SMDT_LG1(EP, ET, 8); } while (0)
  if (dtype == 2) {
    if (epi == 0) SMDT_LG(0, f16); else if (epi == 1) SMDT_LG(1, f16); else SMDT_LG(2, f16);
  } else {
    if (epi == 0) SMDT_LG(0, bf16); else if (epi == 1) SMDT_LG(1, bf16); else SMDT_LG(2, bf16);
  }
#undef SMDT_LG
#undef SMDT_LG1
#undef SMDT_LG4
  return hipGetLastError();
}
