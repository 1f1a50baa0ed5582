// Weight-gradient GEMM with fp32 accumulation into the DDP main_grad:
//     C[n, k] (fp32) += sum_m A[m, n] * B[m, k]       A = dY [M, N], B = X [M, K], bf16 row-major
// (Megatron's gradient-accumulation fusion; /root/reference/3_training_megatron-lm/
// megatron/arguments.py:850-854).
//
// Why a hand-written kernel: the reduction index m (tokens) is the SLOW index of both operands.
// Library GEMMs treat that as the "NT" layout and stage each operand through an LDS transpose;
// on MI355X hipBLASLt's best NT fp32-output kernels reach 0.36-1.0 PF/s on the GPT-2 345M wgrad
// shapes (profiles/r1_attn_dropout/wgrad_variants.jsonl) vs 1.1-1.4 for the same GEMMs with the
// reduction index contiguous. gfx950's ds_read_b64_tr_b16 reads a row-major [m][n] LDS tile by
// COLUMNS, which is exactly an MFMA operand fragment with 8 consecutive m per lane — so both
// operands are staged row-major (plain 16-byte global loads, no transpose anywhere) and read
// transposed from LDS (mfma_tile.h, the same images the flash-attention kernels use).
//
// Structure: 128 x 128 output tile per workgroup (4 waves, 2 x 2, each 64 x 64 = 2 x 2 MFMA
// 32x32x16 accumulators), 64-row m stages double-buffered in LDS (2 x 32 KB) with register
// staging issued before the MFMA work of the current stage (one barrier per stage). Small
// outputs are split along m (split-K) so the grid covers the 256 CUs; split partials are added
// with hardware fp32 atomics, a single split does a plain read-modify-write (deterministic).
// Blocks are remapped so consecutive work items (same split, same n-block) share an XCD's L2.
#include "common.h"
#include "launchers.h"
#include "mfma_tile.h"

namespace smdt {
namespace wg {

using namespace mt;
using G = Geo<128>;
constexpr int BN = 128, BK = 128, BM = kTile;

template <bool ATOMIC>
__global__ __launch_bounds__(256, 2) void wgrad_kernel(const bf16* __restrict__ A, const bf16* __restrict__ B,
                                                     float* __restrict__ C, int M, int N, int K, int ntn,
                                                     int ntk, int m_per_split, int nblocks) {
  __shared__ __attribute__((aligned(16))) char lds[2 * 2 * G::TB];  // [buf][A | B], 64 KB

  // XCD-aware bijective remap (blocks are dispatched round-robin over the 8 XCDs).
  const int orig = blockIdx.x;
  const int xcd = orig & 7, q = nblocks >> 3, r = nblocks & 7;
  const int w = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
  const int tk = w % ntk;
  const int t2 = w / ntk;
  const int tn = t2 % ntn;
  const int split = t2 / ntn;
  const int n0 = tn * BN, k0 = tk * BK;
  const int mstart = split * m_per_split;
  const int mend = min(M, mstart + m_per_split);
  const int nst = (mend - mstart) / BM;

  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, h = lane >> 5;
  const int wr = wv >> 1, wc = wv & 1;  // wave tile: n rows [64 wr, +64), k cols [64 wc, +64)

  Frag<128> fr;
  fr.init(lane);
  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = zero16();

  Stage<128> sa, sb;
  sa.init(N);
  sb.init(K);
  const bf16* Ab = A + (int64_t)mstart * N + n0;
  const bf16* Bb = B + (int64_t)mstart * K + k0;
  if (nst > 0) {
    sa.load(Ab);
    sb.load(Bb);
    sa.store(lds);
    sb.store(lds + G::TB);
  }
  __syncthreads();

  for (int t = 0; t < nst; ++t) {
    const bool more = t + 1 < nst;
    const char* at = lds + (t & 1) * 2 * G::TB;
    const char* bt = at + G::TB;
    if (more) {
      sa.load(Ab + (int64_t)(t + 1) * BM * N);
      sb.load(Bb + (int64_t)(t + 1) * BM * K);
    }
#pragma unroll
    for (int rb = 0; rb < 64; rb += 32) {
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const bf16x8 a0 = fr.trf(at, rb, s, 2 * wr), a1 = fr.trf(at, rb, s, 2 * wr + 1);
        const bf16x8 b0 = fr.trf(bt, rb, s, 2 * wc), b1 = fr.trf(bt, rb, s, 2 * wc + 1);
        acc[0][0] = mfma(a0, b0, acc[0][0]);
        acc[0][1] = mfma(a0, b1, acc[0][1]);
        acc[1][0] = mfma(a1, b0, acc[1][0]);
        acc[1][1] = mfma(a1, b1, acc[1][1]);
      }
    }
    if (more) {
      char* nb = lds + ((t + 1) & 1) * 2 * G::TB;
      sa.store(nb);
      sb.store(nb + G::TB);
    }
    __syncthreads();
  }

  // Epilogue: register r of acc[i][j] is C[n0 + 64 wr + 32 i + acc_row(r, h)][k0 + 64 wc + 32 j + lane&31];
  // the 32 lanes of a half write 32 consecutive fp32 (128 B) per register.
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      float* cp = C + (int64_t)(n0 + 64 * wr + 32 * i) * K + (k0 + 64 * wc + 32 * j + (lane & 31));
#pragma unroll
      for (int r2 = 0; r2 < 16; ++r2) {
        float* p = cp + (int64_t)acc_row(r2, h) * K;
        if constexpr (ATOMIC)
          unsafeAtomicAdd(p, acc[i][j][r2]);
        else
          *p += acc[i][j][r2];
      }
    }
}

}  // namespace wg
}  // namespace smdt

using namespace smdt;

extern "C" int smdt_wgrad_supported(int64_t M, int64_t N, int64_t K) {
  return M > 0 && M % wg::BM == 0 && N % wg::BN == 0 && K % wg::BK == 0 && M < (1ll << 31) &&
         N * K < (1ll << 31);
}

extern "C" hipError_t smdt_wgrad_accumulate(const void* dy, const void* x, float* main_grad, int64_t M,
                                            int64_t N, int64_t K, int max_splits, hipStream_t st) {
  if (!smdt_wgrad_supported(M, N, K)) return hipErrorInvalidValue;
  const int ntn = (int)(N / wg::BN), ntk = (int)(K / wg::BK);
  const int tiles = ntn * ntk;
  // Enough blocks for 2 per CU on 256 CUs, splits of >= 16 stages each.
  int splits = (512 + tiles - 1) / tiles;
  const int max_by_m = (int)(M / (16 * wg::BM));
  if (splits > max_by_m) splits = max_by_m > 0 ? max_by_m : 1;
  if (max_splits > 0 && splits > max_splits) splits = max_splits;
  if (splits < 1) splits = 1;
  int64_t stages = M / wg::BM;
  const int m_per_split = (int)(((stages + splits - 1) / splits) * wg::BM);
  splits = (int)((M + m_per_split - 1) / m_per_split);
  const int nblocks = tiles * splits;
  if (splits > 1)
    hipLaunchKernelGGL((wg::wgrad_kernel<true>), dim3(nblocks), dim3(256), 0, st, (const bf16*)dy, (const bf16*)x,
                       main_grad, (int)M, (int)N, (int)K, ntn, ntk, m_per_split, nblocks);
  else
    hipLaunchKernelGGL((wg::wgrad_kernel<false>), dim3(nblocks), dim3(256), 0, st, (const bf16*)dy, (const bf16*)x,
                       main_grad, (int)M, (int)N, (int)K, ntn, ntk, m_per_split, nblocks);
  return hipGetLastError();
}
