// Per-sample image filters of the Oxford-Pet train augmentation (data/augment.py), fp32 NCHW.
//
//   * depthwise_ps: y[n, c] = x[n, c] (*) k[n] with reflect padding — the per-sample KS x KS
//     kernels of box / motion blur, sharpen and emboss (one kernel per image, shared by its
//     channels). As a torch grouped convolution (groups = N * C) MIOpen ran its naive fp32 NCHW
//     kernel: 5.8 ms of a 31.8 ms ResNet-50 step (profiles/r4_vision/resnet50_last_step_breakdown.txt).
//   * median3: 3 x 3 median per channel with reflect padding (albumentations MedianBlur); torch's
//     unfold + median took 1.4 ms per call (gatherMedian).
//
// Both are memory-bound: a 256-thread block owns a 16 x 16 output tile of one (n, c) plane,
// stages the (16 + KS - 1)^2 input window (reflect-indexed) in LDS once, and every thread then
// reads its KS x KS neighbourhood from LDS. Reference: SURVEY R5 (the reference pipeline's
// albumentations transforms, /root/reference/2_training_oxford-pet_ddp/pytorch_oxford_ddp.py:140-160).
#include "common.h"
#include "launchers.h"

namespace smdt {
namespace aug {

constexpr int kT = 16;  // output tile edge

__device__ __forceinline__ int reflect(int i, int n) {
  i = i < 0 ? -i : i;
  return i >= n ? 2 * n - 2 - i : i;
}

template <int KS>
__device__ __forceinline__ void load_window(const float* __restrict__ xp, float (*tile)[kT + KS], int H, int W,
                                            int y0, int x0) {
  constexpr int P = KS / 2, TS = kT + KS - 1;
  for (int i = threadIdx.x; i < TS * TS; i += 256) {
    const int r = i / TS, c = i - r * TS;
    tile[r][c] = xp[(int64_t)reflect(y0 + r - P, H) * W + reflect(x0 + c - P, W)];
  }
}

template <int KS>
__global__ __launch_bounds__(256) void depthwise_ps_kernel(const float* __restrict__ x, const float* __restrict__ k,
                                                           float* __restrict__ y, int C, int H, int W) {
  __shared__ float tile[kT + KS - 1][kT + KS];
  __shared__ float kk[KS * KS];
  const int plane = blockIdx.z, n = plane / C;
  const int y0 = blockIdx.y * kT, x0 = blockIdx.x * kT;
  load_window<KS>(x + (int64_t)plane * H * W, tile, H, W, y0, x0);
  if (threadIdx.x < KS * KS) kk[threadIdx.x] = k[(int64_t)n * KS * KS + threadIdx.x];
  __syncthreads();
  const int ty = threadIdx.x / kT, tx = threadIdx.x % kT;
  const int oy = y0 + ty, ox = x0 + tx;
  if (oy >= H || ox >= W) return;
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < KS; ++i)
#pragma unroll
    for (int j = 0; j < KS; ++j) s = fmaf(kk[i * KS + j], tile[ty + i][tx + j], s);
  y[(int64_t)plane * H * W + (int64_t)oy * W + ox] = s;
}

__device__ __forceinline__ void cswap(float& a, float& b) {
  const float lo = fminf(a, b), hi = fmaxf(a, b);
  a = lo;
  b = hi;
}

__global__ __launch_bounds__(256) void median3_kernel(const float* __restrict__ x, float* __restrict__ y, int H, int W) {
  __shared__ float tile[kT + 2][kT + 3];
  const int plane = blockIdx.z;
  const int y0 = blockIdx.y * kT, x0 = blockIdx.x * kT;
  load_window<3>(x + (int64_t)plane * H * W, tile, H, W, y0, x0);
  __syncthreads();
  const int ty = threadIdx.x / kT, tx = threadIdx.x % kT;
  const int oy = y0 + ty, ox = x0 + tx;
  if (oy >= H || ox >= W) return;
  float v[9];
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) v[3 * i + j] = tile[ty + i][tx + j];
  // median of 9 by the 19-exchange selection network (Paeth / Devillard): v[4] ends as the median
  cswap(v[1], v[2]); cswap(v[4], v[5]); cswap(v[7], v[8]);
  cswap(v[0], v[1]); cswap(v[3], v[4]); cswap(v[6], v[7]);
  cswap(v[1], v[2]); cswap(v[4], v[5]); cswap(v[7], v[8]);
  cswap(v[0], v[3]); cswap(v[5], v[8]); cswap(v[4], v[7]);
  cswap(v[3], v[6]); cswap(v[1], v[4]); cswap(v[2], v[5]);
  cswap(v[4], v[7]); cswap(v[4], v[2]); cswap(v[6], v[4]);
  cswap(v[4], v[2]);
  y[(int64_t)plane * H * W + (int64_t)oy * W + ox] = v[4];
}

}  // namespace aug
}  // namespace smdt

using namespace smdt;

extern "C" hipError_t smdt_aug_depthwise(const float* x, const float* k, float* y, int N, int C, int H, int W, int ks,
                                         hipStream_t st) {
  if (N <= 0 || C <= 0 || H < ks || W < ks || (int64_t)N * C > 65535) return hipErrorInvalidValue;
  const dim3 grid((unsigned)((W + aug::kT - 1) / aug::kT), (unsigned)((H + aug::kT - 1) / aug::kT), (unsigned)(N * C));
  switch (ks) {
    case 3: hipLaunchKernelGGL(aug::depthwise_ps_kernel<3>, grid, dim3(256), 0, st, x, k, y, C, H, W); break;
    case 5: hipLaunchKernelGGL(aug::depthwise_ps_kernel<5>, grid, dim3(256), 0, st, x, k, y, C, H, W); break;
    case 7: hipLaunchKernelGGL(aug::depthwise_ps_kernel<7>, grid, dim3(256), 0, st, x, k, y, C, H, W); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

extern "C" hipError_t smdt_aug_median3(const float* x, float* y, int planes, int H, int W, hipStream_t st) {
  if (planes <= 0 || planes > 65535 || H < 3 || W < 3) return hipErrorInvalidValue;
  const dim3 grid((unsigned)((W + aug::kT - 1) / aug::kT), (unsigned)((H + aug::kT - 1) / aug::kT), (unsigned)planes);
  hipLaunchKernelGGL(aug::median3_kernel, grid, dim3(256), 0, st, x, y, H, W);
  return hipGetLastError();
}
