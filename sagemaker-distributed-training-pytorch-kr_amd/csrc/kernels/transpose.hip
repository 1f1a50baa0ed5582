// 2-D transpose of a 16-bit (bf16 / fp16) matrix for gfx950: out[C, R] = in[R, C].
//
// Used to feed the dgrad GEMMs in hipBLASLt's faster layout. dX = dY W with W [out, in] row-major
// is a "NN" GEMM on this library build. F.linear(dY, W^T) with a contiguous W^T is "TN", the same
// layout the forward GEMMs run in. At the GPT-2 345M shapes TN is 14-24 % faster
// (benchmarks/bench_dgrad.py, profiles/r2_dgrad_tn/). The transpose has to be cheap next to that
// gain: torch's strided copy moves the 103 MB LM-head weight in 0.47 ms (~0.44 TB/s). This
// kernel is a plain LDS tile transpose. Each 256-thread block reads a 64 x 64 tile with one
// 16-byte load per lane per row segment (8 lanes cover a row's 128 bytes). It writes the tile
// back transposed, also in 16-byte vectors. Rows are padded by 2 elements in LDS, so the column
// reads of the transposed pass spread over the banks.
//
// Weight-gradient / dgrad layout of Megatron's linear layers: SURVEY K14 (GEMMs),
// /root/reference/3_training_megatron-lm/megatron/arguments.py:819-821 (gradient-accumulation fusion).
#include "common.h"
#include "launchers.h"

namespace smdt {

constexpr int kTT = 64;   // tile edge (elements)

__global__ __launch_bounds__(256) void transpose16_kernel(const uint16_t* __restrict__ in,
                                                          uint16_t* __restrict__ out, int R, int C) {
  __shared__ uint16_t t[kTT][kTT + 2];
  const int r0 = blockIdx.x * kTT, c0 = blockIdx.y * kTT;
  // load: 64 rows x 8 vectors of 8 elements; each thread moves 2 vectors
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int v = threadIdx.x + k * 256;
    const int rr = v >> 3, cv = (v & 7) * 8;
    const int r = r0 + rr, c = c0 + cv;
    if (r < R && c < C) {   // C % 8 == 0: a vector is either fully inside or fully outside
      const u16x8 x = __builtin_nontemporal_load(reinterpret_cast<const u16x8*>(in + (int64_t)r * C + c));
#pragma unroll
      for (int j = 0; j < 8; ++j) t[rr][cv + j] = x[j];
    }
  }
  __syncthreads();
  // store: out row c holds column c of the tile, 8 vectors of 8 rows each
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int v = threadIdx.x + k * 256;
    const int cc = v >> 3, rv = (v & 7) * 8;
    const int c = c0 + cc, r = r0 + rv;
    if (c < C && r < R) {   // R % 8 == 0
      u16x8 y;
#pragma unroll
      for (int j = 0; j < 8; ++j) y[j] = t[rv + j][cc];
      *reinterpret_cast<u16x8*>(out + (int64_t)c * R + r) = y;
    }
  }
}

// Row gather with zero fill: dst[r, :] = map[r] >= 0 ? src[map[r], :] : 0, rows of `rb` bytes
// (a multiple of 16). The padding-free SFT micro-batches move attention's inputs between the
// packed [T, W] token rows and the padded [L * b, W] layout with it (models/transformer.py):
// every destination row is written exactly once, so neither a zero fill of the whole padded
// buffer nor a scatter (index_copy / index_add, ~0.6-0.9 TB/s) is needed. One wave per row
// chunk of up to 1 KiB (64 lanes x 16 B), 8 waves per block.
__global__ __launch_bounds__(512) void gather_rows_kernel(const uint8_t* __restrict__ src,
                                                          const int64_t* __restrict__ map,
                                                          uint8_t* __restrict__ dst, int64_t nrows,
                                                          int64_t nsrc, int64_t rb) {
  const int64_t chunks = (rb + 1023) / 1024;
  const int64_t item = (int64_t)blockIdx.x * 8 + (threadIdx.x >> 6);
  if (item >= nrows * chunks) return;
  const int64_t r = item / chunks;
  const int64_t off = (item - r * chunks) * 1024 + (int64_t)(threadIdx.x & 63) * 16;
  if (off >= rb) return;
  const int64_t s = map[r];
  u16x8 v = {};
  if (s >= 0 && s < nsrc) v = __builtin_nontemporal_load(reinterpret_cast<const u16x8*>(src + s * rb + off));
  *reinterpret_cast<u16x8*>(dst + r * rb + off) = v;
}

}  // namespace smdt

using namespace smdt;

extern "C" hipError_t smdt_gather_rows(const void* src, const int64_t* map, void* dst, int64_t nrows,
                                       int64_t nsrc, int64_t row_bytes, hipStream_t st) {
  if (nrows <= 0) return hipSuccess;
  if (row_bytes <= 0 || row_bytes % 16 != 0) return hipErrorInvalidValue;
  const int64_t items = nrows * ((row_bytes + 1023) / 1024);
  const int64_t blocks = (items + 7) / 8;
  if (blocks > 0x7FFFFFFF) return hipErrorInvalidValue;
  hipLaunchKernelGGL(gather_rows_kernel, dim3((unsigned)blocks), dim3(512), 0, st, (const uint8_t*)src, map,
                     (uint8_t*)dst, nrows, nsrc, row_bytes);
  return hipGetLastError();
}

extern "C" hipError_t smdt_transpose16(const void* in, void* out, int64_t R, int64_t C, hipStream_t st) {
  if (R <= 0 || C <= 0 || R % 8 != 0 || C % 8 != 0 || R > (1 << 30) || C > (1 << 30))
    return hipErrorInvalidValue;
  const int64_t gx = (R + kTT - 1) / kTT, gy = (C + kTT - 1) / kTT;
  if (gy > 65535) return hipErrorInvalidValue;
  hipLaunchKernelGGL(transpose16_kernel, dim3((unsigned)gx, (unsigned)gy), dim3(256), 0, st,
                     (const uint16_t*)in, (uint16_t*)out, (int)R, (int)C);
  return hipGetLastError();
}
