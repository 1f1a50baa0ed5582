// Standalone timing of the wgrad MFMA kernel's diagnostic variants (see VAR in
// smdt_amd/csrc/kernels/wgrad_gemm.hip): full kernel, no in-loop DMA, no barrier, no LDS reads.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I smdt_amd/csrc/kernels benchmarks/wgrad_micro.hip -o wgrad_micro
#include "../smdt_amd/csrc/kernels/wgrad_gemm.hip"
#include <cstdio>
#include <vector>

template <int VAR>
float run(const bf16* A, const bf16* B, float* C, int M, int N, int K, int splits, int iters) {
  const int ntn = (N + 255) / 256, ntk = (K + 255) / 256, tiles = ntn * ntk;
  const int stages = M / wg::BM;
  const int mps = ((stages + splits - 1) / splits) * wg::BM;
  splits = (M + mps - 1) / mps;
  const int nb = tiles * splits, gn = ntk <= 4 ? 8 : 4;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int i = 0; i < 3; ++i)
    hipLaunchKernelGGL((wg::wgrad_kernel<false, VAR>), dim3(nb), dim3(512), 0, 0, A, B, C, M, N, K, ntn, ntk, gn, mps, nb);
  hipEventRecord(e0);
  for (int i = 0; i < iters; ++i)
    hipLaunchKernelGGL((wg::wgrad_kernel<false, VAR>), dim3(nb), dim3(512), 0, 0, A, B, C, M, N, K, ntn, ntk, gn, mps, nb);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  return ms * 1000.f / iters;
}

int main() {
  const int M = 16384;
  const int shapes[][2] = {{4096, 4096}, {4096, 1024}, {1024, 4096}, {3072, 1024}, {1024, 1024}};
  bf16 *A, *B;
  float* C;
  hipMalloc(&A, (size_t)M * 4096 * 2);
  hipMalloc(&B, (size_t)M * 4096 * 2);
  hipMalloc(&C, (size_t)4096 * 4096 * 4);
  std::vector<unsigned short> h((size_t)M * 4096);
  unsigned s = 1;
  for (auto& v : h) { s = s * 1664525u + 1013904223u; v = 0x3c00 | ((s >> 16) & 0x3ff) | ((s >> 31) << 15); }
  hipMemcpy(A, h.data(), h.size() * 2, hipMemcpyHostToDevice);
  hipMemcpy(B, h.data(), h.size() * 2, hipMemcpyHostToDevice);
  hipMemset(C, 0, (size_t)4096 * 4096 * 4);
  for (auto& sh : shapes) {
    const int N = sh[0], K = sh[1];
    const double fl = 2.0 * M * N * K;
    const float t0 = run<0>(A, B, C, M, N, K, 1, 10), t1 = run<1>(A, B, C, M, N, K, 1, 10),
                t5 = run<5>(A, B, C, M, N, K, 1, 10), t4 = run<4>(A, B, C, M, N, K, 1, 10);
    printf("N=%d K=%d nosplit: full %.1f us (%.0f TF) | no-DMA %.1f | no-DMA,no-reads %.1f | no-LDS-reads %.1f\n",
           N, K, t0, fl / t0 * 1e-6, t1, t5, t4);
  }
  return 0;
}
