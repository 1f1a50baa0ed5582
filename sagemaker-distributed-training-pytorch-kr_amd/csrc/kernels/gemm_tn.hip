// Forward / dgrad GEMM with fused epilogues (SURVEY K5 + K14):
//     C[m, n] = sum_k A[m, k] * B[n, k]            A [M, K], B [N, K], C [M, N], 16-bit, fp32 accumulate
// i.e. F.linear(x, W) with W in nn.Linear's [out, in] layout (and the dgrad F.linear(dY, W^T) with
// the cached W^T). Epilogues:
//   EPI_NONE       C = acc
//   EPI_BIAS       C = acc + bias[n]
//   EPI_BIAS_GELU  C = acc (the pre-activation the backward needs) and C2 = gelu_tanh(C + bias[n])
//   EPI_DGELU      C = acc * gelu_tanh'(pre[m, n] + bias[n]): the fc2 dgrad with the GeLU backward
//                  of the fc1 activation in its epilogue
// The last two are Megatron's bias_gelu fusion (/root/reference/3_training_megatron-lm/megatron/
// arguments.py:819-821, bias_gelu_fusion=True in 3_training_megatron-lm.ipynb) moved into the fc1
// and fc2-dgrad GEMMs: the separate bias_act_fwd / bias_act_bwd passes over the [tokens, 4h]
// tensors are gone (FusedGeLUMLP, parallel/tensor_parallel.py).
//
// Structure (after cdna_hip_programming.md §5's staged-MFMA GEMM rules; written for gfx950):
//   * persistent: one 512-thread workgroup per CU walks its tiles; blockIdx is remapped so the 32
//     workgroups of an XCD take consecutive tiles, ordered in groups of 8 row blocks (row fastest)
//     so they share few A / B panels in that XCD's L2. The K-stages of ALL its tiles form one
//     stream: the LDS-DMA prefetch runs across tile boundaries;
//   * 256 x 256 output tile, 64-deep K-stages in 2 LDS slots per operand (128-B rows: every DMA
//     request is a whole cache line — 32-deep stages doubled the L2 requests, profiles/r5_gemm_tn/),
//     copied global -> LDS by buffer_load_dwordx4 ... lds with the XOR swizzle (row bits 1..3) on
//     the per-lane SOURCE offset, so the LDS image stays lane-linear and the fragment reads are
//     bank-conflict free;
//   * 8 waves as 2 (m) x 4 (n), each 128 x 64 outputs = 8 x 4 accumulators of
//     v_mfma_f32_16x16x32 (the bf16 shape gfx950 clocks higher on random data than 32x32x16);
//   * a stage is four phases of 16 MFMAs; a phase is a read interval and an MFMA interval between
//     raw s_barriers, and waves 4-7 run one interval behind waves 0-3, so on every SIMD one wave's
//     MFMAs run beside its partner's LDS reads and DMA issue (the wave stagger is worth 8 %);
//   * the operands are swapped in the MFMA (B rows as the A operand): each lane's accumulator
//     holds four consecutive n of one row m; the epilogue stages 16-row blocks through 4 KB of
//     LDS per wave and stores whole 128-B lines (16-byte stores).
//
// Measured on MI355X at the GPT-2 345M step shapes (benchmarks/bench_gemm_tn.py): 0.85-0.92x
// of hipBLASLt's tuned GEMM (MT256x256x64, 4 waves of 128 x 128 with AGPR accumulators, 1.3-1.5
// PFLOP/s) alone, 1.02x (fc1 + bias + GeLU) and 1.05x (fc2 dgrad + GeLU backward) against the
// library GEMM followed by the elementwise pass. A 4-wave 128 x 128-per-wave form of this kernel
// (plain double buffering) measured 0.69 vs 0.47 ms on fc1 and was removed.
#include "activations.h"
#include "common.h"
#include "launchers.h"

#include <type_traits>

namespace smdt {
namespace gt {

constexpr int kT = 256;                  // output tile edge
constexpr int kBK = 64;                  // K per stage
constexpr int kThreads = 512;
constexpr int kRowB = kBK * 2;           // 128-B LDS rows: every DMA request is a whole line
constexpr int kOp = kT * kRowB;          // 32 KB: one operand of a stage
constexpr int kSlot = 2 * kOp;           // A + B
constexpr int kNSlot = 2;
constexpr int kGl = kOp / 2 / 1024 / 8;  // 1-KB DMA wave-instructions per wave per 128-row half (2)
constexpr int kEpiB = 32 * 128;          // per-wave epilogue staging: 2 x 16 rows x 64 columns of 16-bit

enum { EPI_NONE = 0, EPI_BIAS = 1, EPI_BIAS_GELU = 2, EPI_DGELU = 3 };

using lds_void = __attribute__((address_space(3))) void;
using f16x8 = __attribute__((ext_vector_type(8))) _Float16;
using u32x2 = __attribute__((ext_vector_type(2))) unsigned;
using u32x4 = __attribute__((ext_vector_type(4))) unsigned;

template <class E> struct V8;
template <> struct V8<bf16> { using t = bf16x8; };
template <> struct V8<f16> { using t = f16x8; };

__device__ __forceinline__ f32x4 mma(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x4 mma(f16x8 a, f16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

// s_waitcnt vmcnt(n), other counters untouched (gfx9 encoding; n <= 63)
template <int n>
__device__ __forceinline__ void wait_vm() {
  static_assert(n >= 0 && n < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((n & 15) | ((n >> 4) << 14) | (7 << 4) | (15 << 8));
}
template <int a, int b, int c>
__device__ __forceinline__ void wait_vm_sel(int sel) {
  if (sel == 0) wait_vm<a>();
  else if (sel == 1) wait_vm<b>();
  else wait_vm<c>();
}

// 4 fp32 -> 4 x 16-bit packed into 8 bytes
template <class E>
__device__ __forceinline__ u32x2 pack4(float a, float b, float c, float d) {
  using v4 = __attribute__((ext_vector_type(4))) E;
  v4 v = {(E)a, (E)b, (E)c, (E)d};
  return __builtin_bit_cast(u32x2, v);
}
template <class E>
__device__ __forceinline__ void unpack4(u32x2 w, float (&o)[4]) {
  using v4 = __attribute__((ext_vector_type(4))) E;
  v4 v = __builtin_bit_cast(v4, w);
#pragma unroll
  for (int i = 0; i < 4; ++i) o[i] = (float)v[i];
}

// XCD-aware bijective remap: blocks b and b + 8 share an XCD (round-robin dispatch); give each
// XCD a contiguous range.
__device__ __forceinline__ int xcd_remap(int orig, int nblocks) {
  const int xcd = orig & 7, q = nblocks >> 3, rem = nblocks & 7;
  return (xcd < rem ? xcd * (q + 1) : rem * (q + 1) + (xcd - rem) * q) + (orig >> 3);
}

struct Args {
  const void* A;
  const void* B;
  void* C;
  void* C2;
  const void* bias;
  const void* aux;   // EPI_DGELU: the GeLU pre-activation [M, N] (without the bias)
  int M, N, K;
  int ntn;      // N / 256
  int ntm;      // M / 256
  int gm;       // tile order: groups of gm row blocks x all column blocks, rows fastest inside
  int tiles;    // (M / 256) * ntn
  int nt;       // K / 64 (even)
  int skew;     // odd workgroups start this many ~8k-cycle sleeps late (de-phased epilogues), 0 none
};

// Stream cursor: K-step `pos` of this workgroup's tile sequence (wave-uniform).
struct Cur {
  uint64_t a, b;   // byte addresses of the tile's first A row / first B row
  uint32_t k;      // byte offset of the K-step within a row
  int pos, kt, tile;
};

using i32x4 = __attribute__((ext_vector_type(4))) int;

// Buffer resource over [base, base + 2 GB): the DMA's per-lane part is a 32-bit byte offset.
__device__ __forceinline__ i32x4 srd(uint64_t base) {
  return i32x4{(int)(uint32_t)base, (int)(uint32_t)(base >> 32) & 0xffff, 0x7FFFFFFF, 0x00020000};
}

// Two 1-KB LDS-DMA wave-instructions (buffer_load_dwordx4 ... lds) into LDS bytes [lds, lds + 2 KB).
// Inline asm on purpose: hipcc then neither sees an LDS write (no alias waits in front of the
// fragment reads of other slots) nor counts these loads (the counted waits are ours, wait_vm).
// M0 is written and restored inside the statement.
__device__ __forceinline__ void dma2(i32x4 rsrc, uint32_t soff, uint32_t v0, uint32_t v1, uint32_t lds) {
  uint32_t keep;
  asm volatile(
      "s_nop 4\n\t"   // descriptor / offset SGPRs may be fresh from a VALU write (readfirstlane)
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %5\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %1, %3, %4 offen lds\n\t"
      "s_add_u32 m0, m0, 0x400\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %2, %3, %4 offen lds\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(v0), "v"(v1), "s"(rsrc), "s"(soff), "s"(lds)
      : "memory");
}

// One 1-KB LDS-DMA wave-instruction (same form as dma2).
__device__ __forceinline__ void dma1(i32x4 rsrc, uint32_t soff, uint32_t v0, uint32_t lds) {
  uint32_t keep;
  asm volatile(
      "s_nop 4\n\t"
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %4\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %1, %2, %3 offen lds\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(v0), "s"(rsrc), "s"(soff), "s"(lds)
      : "memory");
}


// This lane's index, re-made where it is used: asm volatile is never hoisted out of the tile loop,
// so the epilogue's lane-derived addresses hold no VGPRs across the main loop (the compiler kept
// ~12 precomputed staging / store offsets live through every stage and spilled).
__device__ __forceinline__ int lane_now() {
  int l;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
  return l;
}

// 16-byte store with sc1: the line is written through and DROPPED from the XCD's L2
// (MI355X_MICROARCH.md, store flavours). The output tile is never re-read by this kernel, and a
// plain store keeps it in L2, where 4 MB per XCD per round of tiles evicts the A / B panels the
// other tiles of the round stream from L2.
__device__ __forceinline__ void store16_sc1(void* p, u32x4 v) {
  asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
}

__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(__attribute__((address_space(3))) const char*)p;
}

// VAR: diagnostic ablations for benchmarks/bench_gemm_tn.py only (the library runs VAR = 0):
// bit 0 no in-loop DMA, bit 1 no in-loop fragment reads, bit 2 no wave stagger, bit 3 no stores,
// bit 5 sc1 (L2-bypassing) output stores instead of plain ones; (host) bit 7 / 8 tile groups of 1 / 4
// row blocks instead of 8.
template <class E, int EPI, int VAR = 0>
__global__ __launch_bounds__(kThreads, 1) void gemm_tn_kernel(const Args g) {
  using V = typename V8<E>::t;
  // [A slot 0 | A slot 1 | B slot 0 | B slot 1] 32 KB each, then 4 KB of epilogue staging per
  // wave (160 KB: the whole LDS)
  __shared__ __attribute__((aligned(1024))) char L[kNSlot * kSlot + kThreads / 64 * kEpiB];

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  const int G = gridDim.x;
  const int rb = xcd_remap(blockIdx.x, G);
  if (rb >= g.tiles) return;  // (host sizes G <= tiles; whole workgroup, before any barrier)
  if (g.skew > 0 && (blockIdx.x & 1)) {
    for (int i = 0; i < g.skew; ++i) __builtin_amdgcn_s_sleep(127);
  }
  const int ntile = (g.tiles - rb + G - 1) / G;
  const int total = ntile * g.nt;
  const uint32_t rowb = (uint32_t)g.K * 2;   // bytes per operand row
  const uint64_t Ab = (uint64_t)g.A, Bb = (uint64_t)g.B;

  // ---- fragment reads: row (lane & 15) of a 16-row block, 16-byte chunk 4 ks + (lane >> 4),
  // XOR-swizzled by row bits 1..3 (every ds_read_b128 lane group hits 16 distinct bank slots);
  // the wave's A rows are 128 wr .., its B rows 64 wc ..; LDS = [A slot 0 | A slot 1 | B slot 0 |
  // B slot 1], 32 KB each, so one base register per (operand, ks) reaches both slots within the
  // 16-bit ds_read offset
  const uint32_t l0 = lds_addr(L);
  uint32_t ra[2], rbq[2];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) {
    const uint32_t lo = (lane & 15) * kRowB + 16 * ((4 * ks + (lane >> 4)) ^ ((lane >> 1) & 7));
    ra[ks] = l0 + 128 * wr * kRowB + lo;
    rbq[ks] = l0 + 2 * kOp + 64 * wc * kRowB + lo;
  }
  auto rd = [&](uint32_t addr) -> V {
    return *(const V*)(__attribute__((address_space(3))) const char*)(uintptr_t)addr;
  };

  // ---- per-lane DMA byte offsets: wave-instruction j of a 128-row half writes rows
  // 8 (2 wave + j) + lane / 8, 16-byte slot lane % 8, which holds chunk slot ^ f(row)
  uint32_t voff[kGl];
#pragma unroll
  for (int j = 0; j < kGl; ++j) {
    const int r = 8 * (kGl * wave + j) + (lane >> 3);
    const int c = (lane & 7) ^ ((r >> 1) & 7);
    voff[j] = (uint32_t)r * rowb + 16 * c;
  }
  const uint32_t my_lds = (uint32_t)(kGl * wave) * 1024;
  const uint32_t half_b = 128 * rowb;

  // tile t -> (row block, column block): groups of gm row blocks, row fastest inside a group, so
  // the 32 consecutive tiles an XCD runs together share few A and B panels in its L2
  auto coords = [&](int t, int& tm, int& tn) {
    const int per = g.gm * g.ntn;
    const int grp = t / per, first = grp * g.gm;
    const int gsz = min(g.ntm - first, g.gm);
    const int r = t - grp * per;
    tm = first + r % gsz;
    tn = r / gsz;
  };
  auto tile_base = [&](Cur& c) {
    int tm, tn;
    coords(c.tile, tm, tn);
    c.a = Ab + (uint64_t)tm * kT * rowb;
    c.b = Bb + (uint64_t)tn * kT * rowb;
    c.k = 0;
  };
  auto advance = [&](Cur& c) {
    if (c.pos + 1 >= total) return;  // past the end: keep re-reading the last stage (never consumed)
    ++c.pos;
    if (++c.kt == g.nt) {
      c.kt = 0;
      c.tile += G;
      tile_base(c);
    } else {
      c.k += kBK * 2;
    }
  };
  // DMA of half h (0 A rows 0..127, 1 A rows 128..255, 2 / 3 the same of B) of cursor c's stage
  // into its slot (c.pos & 1)
  auto issue = [&](const Cur& c, int h) {
    dma2(srd(h < 2 ? c.a : c.b), c.k + ((h & 1) ? half_b : 0u), voff[0], voff[1],
         l0 + (uint32_t)(h >> 1) * 2 * kOp + (uint32_t)(c.pos & 1) * kOp + (h & 1) * (kOp / 2) + my_lds);
  };

  f32x4 acc[8][4];
  V fa[8][2], fb[4][2];

  // ---- prologue: stages 0 and 1 in flight, wait for stage 0
  Cur cd;   // cursor of the next DMA (stage u + 2 while stage u runs)
  Cur cb;   // the stage whose B halves the next p0 issues (u + 1)
  {
    Cur c0;
    c0.pos = 0; c0.kt = 0; c0.tile = rb;
    tile_base(c0);
    Cur c1 = c0; advance(c1);
    issue(c0, 0); issue(c0, 1); issue(c0, 2); issue(c0, 3);
    issue(c1, 0); issue(c1, 1);   // (stage 1's B: stage 0's p0)
    cd = c1; advance(cd);
    cb = c1;
  }
  wait_vm<2 * kGl>();   // stage 1's A halves may stay in flight
  __builtin_amdgcn_s_barrier();
  if (wr && !(VAR & 4)) __builtin_amdgcn_s_barrier();   // stagger: waves 4-7 one interval behind

  int otile = rb;
  constexpr int NOUT = EPI == EPI_BIAS_GELU ? 2 : 1;
  constexpr int kStores = 16 * NOUT;   // 16-byte stores per wave of one epilogue
  u32x4 bias_w;                        // 8 bias values of this lane's 16-byte column chunk
  (void)bias_w;
  const uint32_t epi_l = l0 + kNSlot * kSlot + wave * kEpiB;

  auto sync = [&]() {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };
  auto mfma_q = [&](int mh, int ks) {   // 64 x 64 quadrant rows 64 mh .., one 32-deep k-step
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[4 * mh + i][j] = mma(fb[j][ks], fa[4 * mh + i][ks], acc[4 * mh + i][j]);
  };
  // One 64-deep stage in slot SL, four phases of 16 MFMAs each:
  //   p0 reads A rows 0..63 and all 64 B rows of the wave (16 ds_read_b128), DMA of B of stage
  //      u + 1 (the other slot), MFMAs rows 0..63 x k 0..31;
  //   p1 reads A rows 64..127 (8 ds_read_b128), rows 0..63 x k 32..63;
  //   p2 rows 64..127 x k 0..31;
  //   p3 DMA of A of stage u + 2 into this slot (its reads retired two barriers back), wait for
  //      stage u + 1 (stage u + 2's A halves stay in flight, plus the epilogue's stores when this
  //      is a tile's first stage), rows 64..127 x k 32..63.
  // A tile's last stage also issues B of stage u + 2 in p3 (ahead of the epilogue's stores, so the
  // next tile's first waits never cover them), and its first stage then skips the p0 DMA.
  auto stage = [&](auto slc, auto lastc, bool first) {
    constexpr int SL = decltype(slc)::value;
    constexpr bool LAST = decltype(lastc)::value;
    if constexpr (EPI != EPI_NONE && LAST) {
      // this tile's 64 bias values of the wave, by LDS-DMA into the second half of the wave's
      // staging area (lanes 8.. re-load the same 128 bytes): no register held through the stage
      int otm, otn;
      coords(otile, otm, otn);
      dma1(srd((uint64_t)((const E*)g.bias + otn * kT + 64 * wc)), 0u, (uint32_t)(lane_now() & 7) * 16,
           epi_l + 2048);
    }
    // ---------------- p0
    if (!(VAR & 2)) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) fa[i][ks] = rd(ra[ks] + SL * kOp + i * 16 * kRowB);
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) fb[j][ks] = rd(rbq[ks] + SL * kOp + j * 16 * kRowB);
    }
    if (!(VAR & 1) && !first) { issue(cb, 2); issue(cb, 3); }
    sync();
    __builtin_amdgcn_s_setprio(1);
    mfma_q(0, 0);
    __builtin_amdgcn_s_setprio(0);
    sync();
    // ---------------- p1
    if (!(VAR & 2)) {
#pragma unroll
      for (int i = 4; i < 8; ++i)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) fa[i][ks] = rd(ra[ks] + SL * kOp + i * 16 * kRowB);
    }
    sync();
    __builtin_amdgcn_s_setprio(1);
    mfma_q(0, 1);
    __builtin_amdgcn_s_setprio(0);
    sync();
    // ---------------- p2
    sync();
    __builtin_amdgcn_s_setprio(1);
    mfma_q(1, 0);
    __builtin_amdgcn_s_setprio(0);
    sync();
    // ---------------- p3
    if (!(VAR & 1)) { issue(cd, 0); issue(cd, 1); }
    cb = cd;
    if (LAST && !(VAR & 1)) { issue(cb, 2); issue(cb, 3); }
    advance(cd);
    // younger than stage u + 1's last half: stage u + 2's halves issued here
    constexpr int kW = (LAST ? 4 : 2) * kGl;
    if (first) wait_vm<kW + kStores>();
    else wait_vm<kW>();
    sync();
    __builtin_amdgcn_s_setprio(1);
    mfma_q(1, 1);
    __builtin_amdgcn_s_setprio(0);
    sync();
  };

  auto lds_w8 = [&](uint32_t addr, u32x2 v) {
    *(__attribute__((address_space(3))) u32x2*)(uintptr_t)addr = v;
  };
  auto lds_r16 = [&](uint32_t addr) -> u32x4 {
    return *(__attribute__((address_space(3))) const u32x4*)(uintptr_t)addr;
  };
  // bias / activation on 8 consecutive values of one row (chunk rc), o = 0 the first output
  auto finish8 = [&](u32x4 v, int o, u32x4 pv) -> u32x4 {
    if constexpr (EPI == EPI_NONE) {
      return v;
    } else {
      if (EPI == EPI_BIAS_GELU && o == 0) return v;   // the pre-activation
      u32x2 lo = {v[0], v[1]}, hi = {v[2], v[3]};
      if constexpr (EPI == EPI_DGELU) {   // v = d(activation), pv = pre-activation
        u32x2 plo = {pv[0], pv[1]}, phi = {pv[2], pv[3]};
        float x[8], z[8], b[8];
        u32x2 blo = {bias_w[0], bias_w[1]}, bhi = {bias_w[2], bias_w[3]};
        unpack4<E>(lo, *reinterpret_cast<float(*)[4]>(x));
        unpack4<E>(hi, *reinterpret_cast<float(*)[4]>(x + 4));
        unpack4<E>(plo, *reinterpret_cast<float(*)[4]>(z));
        unpack4<E>(phi, *reinterpret_cast<float(*)[4]>(z + 4));
        unpack4<E>(blo, *reinterpret_cast<float(*)[4]>(b));
        unpack4<E>(bhi, *reinterpret_cast<float(*)[4]>(b + 4));
#pragma unroll
        for (int e = 0; e < 8; ++e) x[e] = x[e] * gelu_tanh_grad(z[e] + b[e]);
        const u32x2 ol = pack4<E>(x[0], x[1], x[2], x[3]), oh = pack4<E>(x[4], x[5], x[6], x[7]);
        return u32x4{ol[0], ol[1], oh[0], oh[1]};
      }
      u32x2 blo = {bias_w[0], bias_w[1]}, bhi = {bias_w[2], bias_w[3]};
      float x[8], b[8];
      unpack4<E>(lo, *reinterpret_cast<float(*)[4]>(x));
      unpack4<E>(hi, *reinterpret_cast<float(*)[4]>(x + 4));
      unpack4<E>(blo, *reinterpret_cast<float(*)[4]>(b));
      unpack4<E>(bhi, *reinterpret_cast<float(*)[4]>(b + 4));
#pragma unroll
      for (int e = 0; e < 8; ++e) x[e] = EPI == EPI_BIAS ? x[e] + b[e] : gelu_tanh(x[e] + b[e]);
      const u32x2 ol = pack4<E>(x[0], x[1], x[2], x[3]), oh = pack4<E>(x[4], x[5], x[6], x[7]);
      return u32x4{ol[0], ol[1], oh[0], oh[1]};
    }
  };
  // Epilogue through the wave's 4 KB of LDS, one 16-row block at a time: each lane writes its
  // 4 x 8-byte pieces (4 consecutive n of one row), then reads back 16-byte row chunks, so every
  // global store instruction writes 8 whole 128-byte lines (the accumulator layout alone gives
  // 16 rows x 32 bytes per instruction). The bias is added, and the activation computed, from the
  // rounded 16-bit pre-activation — the arithmetic of the separate bias_act_fwd pass it replaces.
  auto epilogue = [&]() {
    if constexpr (EPI != EPI_NONE) {
      wait_vm<4 * kGl>();   // the bias DMA: older than stage u + 2's 4 halves (and retired already)
      bias_w = lds_r16(epi_l + 2048 + (lane_now() & 7) * 16);
    }
    int otm, otn;
    coords(otile, otm, otn);
    const int64_t N = g.N;
    // EPI_DGELU: the pre-activation rows of the whole wave tile (16 x 16 B per lane, in the
    // read-side layout), issued before any block so their latency overlaps the first blocks
    u32x4 pre_v[8][2];
    if constexpr (EPI == EPI_DGELU) {
      const int ln = lane_now(), rr = ln >> 3, rc = ln & 7;
      const E* pre = (const E*)g.aux + (int64_t)(otm * kT + 128 * wr + rr) * N + otn * kT + 64 * wc + 8 * rc;
#pragma unroll
      for (int k = 0; k < 8; ++k)
#pragma unroll
        for (int h = 0; h < 2; ++h) pre_v[k][h] = *(const u32x4*)(pre + (int64_t)(16 * k + 8 * h) * N);
    } else {
#pragma unroll
      for (int k = 0; k < 8; ++k) pre_v[k][0] = pre_v[k][1] = u32x4{0, 0, 0, 0};
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int ln = lane_now(), r16 = ln & 15, qq = ln >> 4, rr = ln >> 3, rc = ln & 7;
      const uint32_t area = epi_l + (k & 1) * 2048;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const f32x4 v = acc[k][j];
        const int chunk = (2 * j + (qq >> 1)) ^ (r16 & 7);
        lds_w8(area + r16 * 128 + chunk * 16 + (qq & 1) * 8, pack4<E>(v[0], v[1], v[2], v[3]));
      }
      __builtin_amdgcn_sched_barrier(0);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // other lanes' pieces are in place
      __builtin_amdgcn_sched_barrier(0);
      u32x4 rv[2];
      rv[0] = lds_r16(area + rr * 128 + ((rc ^ (rr & 7)) * 16));
      rv[1] = lds_r16(area + (rr + 8) * 128 + ((rc ^ ((rr + 8) & 7)) * 16));
      const int64_t off = (int64_t)(otm * kT + 128 * wr + 16 * k + rr) * N + otn * kT + 64 * wc + 8 * rc;
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int o = 0; o < NOUT; ++o) {
          E* dst = (E*)(o == 0 ? g.C : g.C2) + off + (int64_t)(8 * h) * N;
          const u32x4 w = finish8(rv[h], o + (EPI == EPI_BIAS ? 1 : 0), pre_v[k][h]);
          if constexpr ((VAR & 8) != 0) asm volatile("" ::"v"(w));
          else if constexpr ((VAR & 32) != 0) store16_sc1(dst, w);
          else *(u32x4*)dst = w;
        }
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  using S0 = std::integral_constant<int, 0>;
  using S1 = std::integral_constant<int, 1>;
  using F_ = std::false_type;
  using T_ = std::true_type;

  // tile loop outside, stage pairs inside (nt even: every tile starts in slot 0; the last pair is
  // peeled for the bias load); the DMA cursor runs ahead across the tile boundary on its own
  for (int it = 0; it < ntile; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int kt = 0; kt < g.nt - 2; kt += 2) {
      stage(S0{}, F_{}, kt == 0 && it > 0);
      stage(S1{}, F_{}, false);
    }
    stage(S0{}, F_{}, g.nt == 2 && it > 0);
    stage(S1{}, T_{}, false);
    epilogue();
    otile += G;
  }
  if (!wr && !(VAR & 4)) __builtin_amdgcn_s_barrier();  // matching barrier count for the unstaggered half
  wait_vm<0>();   // trailing re-read DMAs land before the workgroup's LDS is released
}

}  // namespace gt
}  // namespace smdt

using namespace smdt;

extern "C" int smdt_gemm_tn_supported(int64_t M, int64_t N, int64_t K) {
  return M > 0 && N > 0 && M % gt::kT == 0 && N % gt::kT == 0 && K % (2 * gt::kBK) == 0 &&
         M * K < (1ll << 31) && N * K < (1ll << 31) && (M / gt::kT) * (N / gt::kT) < (1ll << 30);
}

static int gt_num_cus() {
  static int n = [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0)
      v = 256;
    return v;
  }();
  return n;
}

extern "C" hipError_t smdt_gemm_tn(int dtype, int epi, const void* a, const void* b, void* c, void* c2,
                                   const void* bias, const void* aux, int64_t M, int64_t N, int64_t K,
                                   int max_blocks, hipStream_t st) {
  return smdt_gemm_tn_var(dtype, epi, a, b, c, c2, bias, aux, M, N, K, max_blocks, 0, st);
}

extern "C" hipError_t smdt_gemm_tn_var(int dtype, int epi, const void* a, const void* b, void* c, void* c2,
                                       const void* bias, const void* aux, int64_t M, int64_t N, int64_t K,
                                       int max_blocks, int var, hipStream_t st) {
  if (dtype != 1 && dtype != 2) return hipErrorInvalidValue;
  if (!smdt_gemm_tn_supported(M, N, K)) return hipErrorInvalidValue;
  if (epi < 0 || epi > 3 || (epi >= 1 && !bias) || (epi == 2 && !c2) || (epi == 3 && !aux)) return hipErrorInvalidValue;
  gt::Args g;
  g.A = a; g.B = b; g.C = c; g.C2 = c2; g.bias = bias; g.aux = aux;
  g.M = (int)M; g.N = (int)N; g.K = (int)K;
  g.ntn = (int)(N / gt::kT);
  g.ntm = (int)(M / gt::kT);
  g.gm = (var & 128) ? 1 : (var & 256) ? 4 : 8;   // 8 measured best (fc1 / fc2 / qkv shapes)
  g.tiles = (int)(M / gt::kT) * g.ntn;
  g.nt = (int)(K / gt::kBK);   // stages of 64, even
  g.skew = 0;
  if (var & 64) {   // diagnostic: odd workgroups start about half a tile late (~2k cycles per stage, 8k per sleep)
    g.skew = g.nt / 8 > 0 ? g.nt / 8 : 1;
    var &= ~64;
  }
  if (var & 1024) {   // diagnostic: odd workgroups start about a quarter tile late
    g.skew = g.nt / 16 > 0 ? g.nt / 16 : 1;
    var &= ~1024;
  }
  int grid = gt_num_cus();
  if (max_blocks > 0 && max_blocks < grid) grid = max_blocks;
  if (grid > g.tiles) grid = g.tiles;
#define SMDT_GT(E, P) hipLaunchKernelGGL((gt::gemm_tn_kernel<E, P>), dim3(grid), dim3(gt::kThreads), 0, st, g)
#define SMDT_GTV(V) hipLaunchKernelGGL((gt::gemm_tn_kernel<bf16, 0, V>), dim3(grid), dim3(gt::kThreads), 0, st, g)
  if (var != 0) {   // diagnostic ablations: bf16, no epilogue
    if (dtype != 1 || epi != 0) return hipErrorInvalidValue;
    switch (var) {
      case 1: SMDT_GTV(1); break;
      case 2: SMDT_GTV(2); break;
      case 3: SMDT_GTV(3); break;
      case 4: SMDT_GTV(4); break;
      case 8: SMDT_GTV(8); break;
      case 11: SMDT_GTV(11); break;
      case 32: SMDT_GTV(32); break;
      case 128: SMDT_GTV(0); break;    // (tile order only: g.gm)
      case 256: SMDT_GTV(0); break;
      default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
  }
#undef SMDT_GTV
  if (dtype == 1) {
    if (epi == 0) SMDT_GT(bf16, 0); else if (epi == 1) SMDT_GT(bf16, 1); else if (epi == 2) SMDT_GT(bf16, 2); else SMDT_GT(bf16, 3);
  } else {
    if (epi == 0) SMDT_GT(f16, 0); else if (epi == 1) SMDT_GT(f16, 1); else if (epi == 2) SMDT_GT(f16, 2); else SMDT_GT(f16, 3);
  }
#undef SMDT_GT
  return hipGetLastError();
}
