// Forward / dgrad GEMM with fused epilogues (SURVEY K5 + K14):
//     C[m, n] = sum_k A[m, k] * B[n, k]            A [M, K], B [N, K], C [M, N], 16-bit, fp32 accumulate
// i.e. F.linear(x, W) with W in nn.Linear's [out, in] layout (and the dgrad F.linear(dY, W^T) with
// the cached W^T). Epilogues:
//   EPI_NONE       C = acc
//   EPI_BIAS       C = acc + bias[n]
//   EPI_BIAS_GELU  C = acc (the pre-activation the backward needs) and C2 = gelu_tanh(acc + bias[n])
//                  — Megatron's bias_gelu fusion (/root/reference/3_training_megatron-lm/megatron/
//                  arguments.py:819-821, bias_gelu_fusion=True in 3_training_megatron-lm.ipynb)
//                  moved into the fc1 GEMM: the [tokens, 4h] pre-activation is never re-read.
//
// Structure (after cdna_hip_programming.md §5's staged-MFMA GEMM rules; written for gfx950):
//   * persistent: one 512-thread workgroup per CU walks its tiles (blockIdx remapped so the 32
//     workgroups of an XCD take consecutive tiles, n fastest: they share A rows / B panels in that
//     XCD's L2). The K-stages of ALL its tiles form one stream: the LDS-DMA prefetch runs across
//     tile boundaries, so a tile's epilogue (registers -> global stores, no LDS) overlaps the next
//     tile's operand loads;
//   * 256 x 256 output tile, 32-deep K-stages in a ring of 4 LDS slots (A 256 x 32 + B 256 x 32,
//     32 KB each, 128 KB), copied global -> LDS by buffer_load_dwordx4 ... lds. 64-B rows, 16-B
//     chunks XOR-swizzled by row bits 2..3 (f = -(r >> 2) & 3: every ds_read_b128 lane group hits 16
//     distinct bank slots); the swizzle is applied to the per-lane SOURCE offset, the LDS image
//     stays lane-linear;
//   * 8 waves as 2 (m) x 4 (n), each 128 x 64 outputs = 8 x 4 accumulators of
//     v_mfma_f32_16x16x32 (the bf16 shape gfx950 clocks higher on random data than 32x32x16);
//   * a stage is two phases: (a) read A rows 0..63 of the wave + all its 64 B rows, 16 MFMAs;
//     (b) read A rows 64..127, 16 MFMAs with the B fragments still in registers. A phase is a read
//     interval (ds_reads + one half of a stage's DMA + at most one counted vmcnt) and an MFMA
//     interval, separated by raw s_barriers; waves 4-7 run one barrier behind waves 0-3, so on
//     every SIMD one wave's MFMAs run beside its partner's LDS reads and DMA issue;
//   * the operands are swapped in the MFMA (B rows as the A operand): each lane's accumulator
//     then holds FOUR CONSECUTIVE n of one row m, stored as one 8-byte write per accumulator.
//
// Prefetch schedule (stage u of the stream, slot u % 4): phase (a) issues B of stage u + 2,
// phase (b) issues A of stage u + 3, and phase (b) waits for stage u + 1 (vmcnt(6): the three
// younger halves stay in flight; +the epilogue's stores / bias loads where they sit between).
// A slot is refilled two phases after its last read (b of stage u -> A of u + 4 at b of u + 1),
// the distance that covers the staggered half's reads (retired by its lgkmcnt one barrier later).
#include "activations.h"
#include "common.h"
#include "launchers.h"

#include <type_traits>

namespace smdt {
namespace gt {

constexpr int kT = 256;                  // output tile edge
constexpr int kBK = 32;                  // K per stage
constexpr int kThreads = 512;
constexpr int kRowB = kBK * 2;           // 64-B LDS rows
constexpr int kOp = kT * kRowB;          // 16 KB: one operand of a stage
constexpr int kSlot = 2 * kOp;           // A + B
constexpr int kNSlot = 4;
constexpr int kGl = kOp / 1024 / 8;      // 1-KB DMA wave-instructions per wave per operand (2)
constexpr int kEpiB = 32 * 128;          // per-wave epilogue staging: 2 x 16 rows x 64 columns of 16-bit

enum { EPI_NONE = 0, EPI_BIAS = 1, EPI_BIAS_GELU = 2 };

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
  int M, N, K;
  int ntn;      // N / 256
  int tiles;    // (M / 256) * ntn
  int nt;       // K / 32 (a multiple of 4)
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

// Loads hidden from hipcc's wait bookkeeping (retired by our own counted wait + a "+v" statement
// naming the destination, so the compiler cannot touch the register before the data lands).
__device__ __forceinline__ void load16_hidden(u32x4& d, const void* p) {
  asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(d) : "v"(p) : "memory");
}
// retires a hidden load that is older than the 2 youngest DMA halves (4 wave-instructions)
__device__ __forceinline__ void wait_reg4(u32x4& a) {
  asm volatile("s_waitcnt vmcnt(4)" : "+v"(a) :: "memory");
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
// bit 5 plain (L2-allocating) output stores instead of sc1.
template <class E, int EPI, bool TRICKLE, int VAR = 0>
__global__ __launch_bounds__(kThreads, 1) void gemm_tn_kernel(const Args g) {
  using V = typename V8<E>::t;
  // [slot][A 16 KB | B 16 KB] x 4, then 4 KB of epilogue staging per wave (160 KB: the whole LDS)
  __shared__ __attribute__((aligned(1024))) char L[kNSlot * kSlot + kThreads / 64 * kEpiB];

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  const int G = gridDim.x;
  const int rb = xcd_remap(blockIdx.x, G);
  if (rb >= g.tiles) return;  // (host sizes G <= tiles; whole workgroup, before any barrier)
  const int ntile = (g.tiles - rb + G - 1) / G;
  const int total = ntile * g.nt;
  const uint32_t rowb = (uint32_t)g.K * 2;   // bytes per operand row
  const uint64_t Ab = (uint64_t)g.A, Bb = (uint64_t)g.B;

  // ---- fragment read bases: row (lane & 15) of a 16-row block, chunk lane >> 4 swizzled by
  // f(row) = -(row >> 2) & 3; the wave's A rows are 128 wr .., its B rows 64 wc ..
  const uint32_t l0 = lds_addr(L);
  const uint32_t lo = (lane & 15) * kRowB + 16 * ((lane >> 4) ^ ((4 - ((lane >> 2) & 3)) & 3));
  const uint32_t ra = l0 + 128 * wr * kRowB + lo;
  const uint32_t rbq = l0 + kOp + 64 * wc * kRowB + lo;
  // slots 2, 3 lie beyond the 16-bit ds_read offset field: their own base registers (opaque, so
  // the compiler does not re-derive one address register per fragment from the slot 0 base)
  uint32_t ra_hi = ra + 2 * kSlot, rb_hi = rbq + 2 * kSlot;
  asm volatile("" : "+v"(ra_hi), "+v"(rb_hi));
  auto rd = [&](uint32_t addr) -> V {
    return *(const V*)(__attribute__((address_space(3))) const char*)(uintptr_t)addr;
  };

  // ---- per-lane DMA byte offsets: wave-instruction j writes rows 16 (2 wave + j) + lane / 4,
  // slot lane % 4, which holds chunk slot ^ f(row)
  uint32_t voff[kGl];
#pragma unroll
  for (int j = 0; j < kGl; ++j) {
    const int r = 16 * (kGl * wave + j) + (lane >> 2);
    const int c = (lane & 3) ^ ((4 - ((r >> 2) & 3)) & 3);
    voff[j] = (uint32_t)r * rowb + 16 * c;
  }
  const uint32_t my_lds = (uint32_t)(kGl * wave) * 1024;

  auto tile_base = [&](Cur& c) {
    const int tm = c.tile / g.ntn, tn = c.tile - tm * g.ntn;
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
  // DMA of operand op (0 A, 1 B) of cursor c's stage into its ring slot (c.pos % 4)
  auto issue = [&](const Cur& c, int op) {
    dma2(srd(op ? c.b : c.a), c.k, voff[0], voff[1],
         l0 + (uint32_t)(c.pos & (kNSlot - 1)) * kSlot + op * kOp + my_lds);
  };

  f32x4 acc[8][4];
  V fa[4], fb[4];
  if constexpr ((VAR & 2) != 0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) { fa[i] = rd(ra + i * 1024); fb[i] = rd(rbq + i * 1024); }
  }

  // ---- prologue: A / B of stages 0, 1 and A of stage 2 in flight; wait for stage 0
  Cur cb, ca;  // cursors of the next B issue (stage u + 2) and the next A issue (stage u + 3)
  {
    Cur c0;
    c0.pos = 0; c0.kt = 0; c0.tile = rb;
    tile_base(c0);
    Cur c1 = c0; advance(c1);
    Cur c2 = c1; advance(c2);
    issue(c0, 0); issue(c0, 1); issue(c1, 0); issue(c1, 1); issue(c2, 0);
    cb = c2;
    ca = c2; advance(ca);
  }
  wait_vm<3 * kGl>();   // the 3 youngest halves may stay in flight
  __builtin_amdgcn_s_barrier();
  if (wr && !(VAR & 4)) __builtin_amdgcn_s_barrier();   // stagger: waves 4-7 one interval behind

  int otile = rb;
  constexpr int NOUT = EPI == EPI_BIAS_GELU ? 2 : 1;
  // Epilogue, half trickled: rows 0..63 of the wave's finished tile are stored at once, rows
  // 64..127 wait as packed 16-bit values (pend, 32 VGPRs: all 128 rows would spill) and are
  // stored over the NEXT tile's first 4 stages, one 16-row block per stage: each lane writes its
  // 4 x 8-byte pieces (4 consecutive n of one row) into the wave's LDS staging, reads back 16-byte
  // row chunks, and every global store instruction writes 8 whole 128-byte lines. (Stored at the
  // tile's end instead, the 256 workgroups — which finish their tiles together — put a 32 MB
  // burst on HBM and the next tile's operand DMA queued behind it: +25 % on a K = 1024 GEMM.)
  // The bias is added, and the activation computed, from the rounded 16-bit pre-activation at
  // store time — the same arithmetic as the separate bias_act_fwd pass it replaces.
  u32x2 pend[4][4];   // blocks 4..7 of the finished tile
  u32x4 bias_w;              // 8 bias values of this lane's 16-byte column chunk
  bool has_pend = false;
  int ptile = 0;             // tile of the pending values
  const uint32_t epi_l = l0 + kNSlot * kSlot + wave * kEpiB;

  auto sync = [&]() {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };
  auto lds_w8 = [&](uint32_t addr, u32x2 v) {
    *(__attribute__((address_space(3))) u32x2*)(uintptr_t)addr = v;
  };
  auto lds_r16 = [&](uint32_t addr) -> u32x4 {
    return *(__attribute__((address_space(3))) const u32x4*)(uintptr_t)addr;
  };
  // bias / activation on 8 consecutive values of one row (chunk rc)
  auto finish8 = [&](u32x4 v, int o) -> u32x4 {
    if constexpr (EPI == EPI_NONE) {
      return v;
    } else {
      if (EPI == EPI_BIAS_GELU && o == 0) return v;
      u32x2 lo = {v[0], v[1]}, hi = {v[2], v[3]};
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
  // Store 8 rows (half h of pending block k) from the staging area: NOUT store instructions.
  auto block_rows = [&](int k, int h, u32x4 v) {
    const int ln = lane_now(), rr = ln >> 3, rc = ln & 7;   // read side: row (+ 8 h), 16-byte chunk
    const int ptm = ptile / g.ntn, ptn = ptile - ptm * g.ntn;
    const int64_t N = g.N;
    const int64_t off = (int64_t)(ptm * kT + 128 * wr + 16 * k + 8 * h + rr) * N + ptn * kT + 64 * wc + 8 * rc;
#pragma unroll
    for (int o = 0; o < NOUT; ++o) {
      E* dst = (E*)(o == 0 ? g.C : g.C2) + off;
      const u32x4 w = finish8(v, o + (EPI == EPI_BIAS ? 1 : 0));
      if constexpr ((VAR & 8) != 0) asm volatile("" ::"v"(w));
      else if constexpr ((VAR & 32) != 0) *(u32x4*)dst = w;
      else store16_sc1(dst, w);
    }
  };
  // 16-row block k (4 packed pieces per lane) -> the wave's staging area (half k & 1), read back
  // as two 8-row halves
  auto stage_block = [&](int k, const u32x2 (&pc)[4], u32x4& r0, u32x4& r1) {
    // write side: row r16 of the block, columns 16 j + 4 qq; read side: row rr (+ 8), chunk rc
    const int ln = lane_now(), r16 = ln & 15, qq = ln >> 4, rr = ln >> 3, rc = ln & 7;
    const uint32_t area = epi_l + (k & 1) * 2048;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int chunk = (2 * j + (qq >> 1)) ^ (r16 & 7);
      lds_w8(area + r16 * 128 + chunk * 16 + (qq & 1) * 8, pc[j]);
    }
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // other lanes' pieces are in place
    __builtin_amdgcn_sched_barrier(0);
    r0 = lds_r16(area + rr * 128 + ((rc ^ (rr & 7)) * 16));
    r1 = lds_r16(area + (rr + 8) * 128 + ((rc ^ ((rr + 8) & 7)) * 16));
  };
  u32x4 held;   // second half of the block staged in phase (a), stored in phase (b)

  // One stage. SK: trickle window stage (0..3: store pending block 4 + SK; 4: the stage after
  // the window; -1: none). LAST: the tile's last stage (bias load). The phase (b) wait leaves the 3
  // younger DMA halves in flight plus every store / bias load issued after the awaited half.
  auto stage = [&](auto slotc, auto skc, auto lastc) {
    constexpr int slot = decltype(slotc)::value;
    constexpr int SK = decltype(skc)::value;
    constexpr bool LAST = decltype(lastc)::value;
    constexpr uint32_t so = (slot & 1) * kSlot;
    const uint32_t ra_s = slot < 2 ? ra : ra_hi;
    const uint32_t rb_s = slot < 2 ? rbq : rb_hi;
    if constexpr (EPI != EPI_NONE && LAST) {   // this tile's bias for the read-side chunk
      const int otn = otile - (otile / g.ntn) * g.ntn;
      load16_hidden(bias_w, (const E*)g.bias + otn * kT + 64 * wc + 8 * (lane_now() & 7));
    }
    // ---------------- phase (a): A rows 0..63 x B rows 0..63 of the wave
#pragma unroll
    for (int i = 0; i < 4; ++i) if (!(VAR & 2)) fa[i] = rd(ra_s + so + i * 16 * kRowB);
#pragma unroll
    for (int j = 0; j < 4; ++j) if (!(VAR & 2)) fb[j] = rd(rb_s + so + j * 16 * kRowB);
    if constexpr (SK >= 0 && SK < 4) {
      if (has_pend) {
        u32x4 r0;
        stage_block(4 + SK, pend[SK], r0, held);
        block_rows(4 + SK, 0, r0);
      }
    }
    if (!(VAR & 1)) issue(cb, 1);
    advance(cb);
    sync();
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = mma(fb[j], fa[i], acc[i][j]);
    __builtin_amdgcn_s_setprio(0);
    sync();
    // ---------------- phase (b): A rows 64..127
#pragma unroll
    for (int i = 0; i < 4; ++i) if (!(VAR & 2)) fa[i] = rd(ra_s + so + (64 + i * 16) * kRowB);
    if constexpr (SK >= 0 && SK < 4) {
      if (has_pend) block_rows(4 + SK, 1, held);
    }
    if (!(VAR & 1)) issue(ca, 0);
    advance(ca);
    // stores younger than the awaited half (B of the next stage, issued in phase (a) of the
    // previous stage, after that phase's stores): phase (b) of the previous stage, (a) and (b) of
    // this one — and, at the first stage, the 8 direct stores of the tile's retirement
    // (SK 9: first stage after a retirement that stored all 8 blocks at once)
    constexpr int kSt = NOUT * (SK == 0 ? 10 : (SK > 0 && SK < 4) ? 3 : SK == 4 ? 1 : SK == 9 ? 16 : 0);
    constexpr int kW = 3 * kGl + ((EPI != EPI_NONE && LAST) ? 1 : 0);
    if (kSt > 0 && has_pend) wait_vm<kW + kSt>();
    else wait_vm<kW>();
    sync();
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[4 + i][j] = mma(fb[j], fa[i], acc[4 + i][j]);
    __builtin_amdgcn_s_setprio(0);
    sync();
  };

  // finished tile: blocks 0..3 stored now, blocks 4..7 -> pend (16-bit pre-activation / product);
  // without TRICKLE (fewer than 12 stages per tile) all 8 blocks are stored now
  auto retire_tile = [&]() {
    if constexpr (EPI != EPI_NONE) wait_reg4(bias_w);   // older than the last stage's 2 DMA halves
    ptile = otile;
#pragma unroll
    for (int k = 0; k < (TRICKLE ? 4 : 8); ++k) {
      u32x2 pc[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const f32x4 v = acc[k][j];
        pc[j] = pack4<E>(v[0], v[1], v[2], v[3]);
        acc[k][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
      u32x4 r0, r1;
      stage_block(k, pc, r0, r1);
      block_rows(k, 0, r0);
      block_rows(k, 1, r1);
      __builtin_amdgcn_sched_barrier(0);
    }
    if constexpr (TRICKLE) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const f32x4 v = acc[4 + i][j];
          pend[i][j] = pack4<E>(v[0], v[1], v[2], v[3]);
          acc[4 + i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
    }
    has_pend = true;
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using I2 = std::integral_constant<int, 2>;
  using I3 = std::integral_constant<int, 3>;
  using NO = std::integral_constant<int, -1>;
  using F_ = std::false_type;
  using T_ = std::true_type;

#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // tile loop outside, stages inside (nt % 4 == 0 and nt >= 12: every tile starts on slot 0; the
  // first 8 stages are peeled for the store window, the last 4 for the bias load); the DMA
  // cursors run ahead across the tile boundary on their own
  for (int it = 0; it < ntile && TRICKLE; ++it) {
    stage(I0{}, std::integral_constant<int, 0>{}, F_{});
    stage(I1{}, std::integral_constant<int, 1>{}, F_{});
    stage(I2{}, std::integral_constant<int, 2>{}, F_{});
    stage(I3{}, std::integral_constant<int, 3>{}, F_{});
    stage(I0{}, std::integral_constant<int, 4>{}, F_{});
    stage(I1{}, NO{}, F_{});
    stage(I2{}, NO{}, F_{});
    stage(I3{}, NO{}, F_{});
    for (int kt = 8; kt < g.nt - 4; kt += 4) {
      stage(I0{}, NO{}, F_{});
      stage(I1{}, NO{}, F_{});
      stage(I2{}, NO{}, F_{});
      stage(I3{}, NO{}, F_{});
    }
    stage(I0{}, NO{}, F_{});
    stage(I1{}, NO{}, F_{});
    stage(I2{}, NO{}, F_{});
    stage(I3{}, NO{}, T_{});
    retire_tile();
    otile += G;
  }
  using S9 = std::integral_constant<int, 9>;
  for (int it = 0; it < ntile && !TRICKLE; ++it) {
    if (g.nt == 4) {
      stage(I0{}, S9{}, F_{});
      stage(I1{}, NO{}, F_{});
      stage(I2{}, NO{}, F_{});
      stage(I3{}, NO{}, T_{});
    } else {
      stage(I0{}, S9{}, F_{});
      stage(I1{}, NO{}, F_{});
      stage(I2{}, NO{}, F_{});
      stage(I3{}, NO{}, F_{});
      for (int kt = 4; kt < g.nt - 4; kt += 4) {
        stage(I0{}, NO{}, F_{});
        stage(I1{}, NO{}, F_{});
        stage(I2{}, NO{}, F_{});
        stage(I3{}, NO{}, F_{});
      }
      stage(I0{}, NO{}, F_{});
      stage(I1{}, NO{}, F_{});
      stage(I2{}, NO{}, F_{});
      stage(I3{}, NO{}, T_{});
    }
    retire_tile();
    otile += G;
  }
  // the last tile's pending half: nothing left to hide it behind
#pragma unroll
  for (int k = 0; k < (TRICKLE ? 4 : 0); ++k) {
    u32x4 r0, r1;
    stage_block(4 + k, pend[k], r0, r1);
    block_rows(4 + k, 0, r0);
    block_rows(4 + k, 1, r1);
  }
  if (!wr && !(VAR & 4)) __builtin_amdgcn_s_barrier();  // matching barrier count for the unstaggered half
  wait_vm<0>();   // trailing re-read DMAs land before the workgroup's LDS is released
}

}  // namespace gt
}  // namespace smdt

using namespace smdt;

extern "C" int smdt_gemm_tn_supported(int64_t M, int64_t N, int64_t K) {
  return M > 0 && N > 0 && M % gt::kT == 0 && N % gt::kT == 0 && K % (4 * gt::kBK) == 0 &&
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
                                   const void* bias, int64_t M, int64_t N, int64_t K, int max_blocks,
                                   hipStream_t st) {
  return smdt_gemm_tn_var(dtype, epi, a, b, c, c2, bias, M, N, K, max_blocks, 0, st);
}

extern "C" hipError_t smdt_gemm_tn_var(int dtype, int epi, const void* a, const void* b, void* c, void* c2,
                                       const void* bias, int64_t M, int64_t N, int64_t K, int max_blocks,
                                       int var, hipStream_t st) {
  if (dtype != 1 && dtype != 2) return hipErrorInvalidValue;
  if (!smdt_gemm_tn_supported(M, N, K)) return hipErrorInvalidValue;
  if (epi < 0 || epi > 2 || (epi >= 1 && !bias) || (epi == 2 && !c2)) return hipErrorInvalidValue;
  gt::Args g;
  g.A = a; g.B = b; g.C = c; g.C2 = c2; g.bias = bias;
  g.M = (int)M; g.N = (int)N; g.K = (int)K;
  g.ntn = (int)(N / gt::kT);
  g.tiles = (int)(M / gt::kT) * g.ntn;
  g.nt = (int)(K / gt::kBK);   // stages of 32, a multiple of 4
  int grid = gt_num_cus();
  if (max_blocks > 0 && max_blocks < grid) grid = max_blocks;
  if (grid > g.tiles) grid = g.tiles;
  // half-trickled epilogue from 12 stages per tile (its 4-stage store window + peeled groups)
  const bool tr = g.nt >= 12 && !(var & 16);
#define SMDT_GT(E, P)                                                                                      \
  do {                                                                                                     \
    if (tr) hipLaunchKernelGGL((gt::gemm_tn_kernel<E, P, true>), dim3(grid), dim3(gt::kThreads), 0, st, g); \
    else hipLaunchKernelGGL((gt::gemm_tn_kernel<E, P, false>), dim3(grid), dim3(gt::kThreads), 0, st, g);   \
  } while (0)
#define SMDT_GTV(V) hipLaunchKernelGGL((gt::gemm_tn_kernel<bf16, 0, true, V>), dim3(grid), dim3(gt::kThreads), 0, st, g)
  if (var != 0) {   // diagnostic ablations: bf16, no epilogue
    if (dtype != 1 || epi != 0) return hipErrorInvalidValue;
    switch (var) {
      case 16: SMDT_GT(bf16, 0); break;   // every block stored at the tile's end (no trickle)
      case 1: SMDT_GTV(1); break;
      case 2: SMDT_GTV(2); break;
      case 3: SMDT_GTV(3); break;
      case 4: SMDT_GTV(4); break;
      case 8: SMDT_GTV(8); break;
      case 11: SMDT_GTV(11); break;
      case 32: SMDT_GTV(32); break;
      default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
  }
#undef SMDT_GTV
  if (dtype == 1) {
    if (epi == 0) SMDT_GT(bf16, 0); else if (epi == 1) SMDT_GT(bf16, 1); else SMDT_GT(bf16, 2);
  } else {
    if (epi == 0) SMDT_GT(f16, 0); else if (epi == 1) SMDT_GT(f16, 1); else SMDT_GT(f16, 2);
  }
#undef SMDT_GT
  return hipGetLastError();
}
