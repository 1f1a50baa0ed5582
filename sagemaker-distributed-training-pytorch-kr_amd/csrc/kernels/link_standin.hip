// Paced link stand-in for single-GPU rank emulation (comm/loopback.py).
//
// An emulated TP rank used to replace each TP-pair exchange with an in-line copy: it paid neither
// the transfer time of the real links nor the CUs the real transfer engine occupies, so it could
// not show how much of an exchange the rank's compute hides. This kernel stands in for the relay
// engine's exchange (comm/relay.py, csrc/kernels/xgmi_relay.hip) on the loopback group's side
// stream:
//   * it runs on the same number of workgroups as the relay kernel (64 x 512 threads on an
//     8-GPU node: 2 directions x 8 parts x 4 blocks), so it takes those CUs away from the
//     concurrently running compute, as the relay does;
//   * it copies send -> recv (the receiving side's memory traffic);
//   * it does not finish before `ns` nanoseconds have passed since its first workgroup started
//     (the modelled link time of the message, e.g. 131 us per 33.6 MB for the relay at 64 GB/s
//     per link and direction, docs/XGMI.md), spinning with s_sleep on the constant 100 MHz
//     clock (s_memrealtime), like the relay's blocks that poll their partner's flags.
// Every workgroup exits after a bounded time: the deadline is at most `ns` after its own start.
#include "common.h"
#include "launchers.h"

namespace smdt {
namespace link {

constexpr int kThreads = 512;

__global__ __launch_bounds__(kThreads) void paced_copy_kernel(const uint4* __restrict__ src, uint4* __restrict__ dst,
                                                               int64_t n16, uint64_t ticks) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  const int64_t stride = (int64_t)gridDim.x * kThreads;
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n16; i += stride) dst[i] = src[i];
  // pace: hold the CU until the modelled transfer time has passed (bounded by `ticks`)
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(32);
}

}  // namespace link
}  // namespace smdt

extern "C" hipError_t smdt_paced_copy(const void* src, void* dst, int64_t nbytes, int blocks, int64_t ns,
                                      hipStream_t st) {
  if (nbytes < 0 || nbytes % 16 != 0 || blocks <= 0 || blocks > 1024 || ns < 0 || ns > 100000000)
    return hipErrorInvalidValue;
  const uint64_t ticks = (uint64_t)((ns + 9) / 10);   // s_memrealtime: 100 MHz
  hipLaunchKernelGGL(smdt::link::paced_copy_kernel, dim3(blocks), dim3(smdt::link::kThreads), 0, st,
                     (const uint4*)src, (uint4*)dst, nbytes / 16, ticks);
  return hipGetLastError();
}
