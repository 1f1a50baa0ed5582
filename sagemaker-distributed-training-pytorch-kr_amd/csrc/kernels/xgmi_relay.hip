// Multi-path pairwise exchange over xGMI (docs/XGMI.md): the tensor-
// parallel pair of a TP=2 layout swaps a sequence chunk per ring step (tensor_parallel.ag_ring /
// rs_ring). Between two MI355X GPUs there is ONE direct xGMI link (~64-77 GB/s per direction);
// the other 6 links of each GPU sit idle during that swap. Here a message from rank f to its
// partner g is cut into W equal parts: 2 go straight into g's staging buffer, the other W - 2 are
// written into the staging buffers of the W - 2 other GPUs of the node ("relays") and g pulls them
// from there. A relay runs no code: its HBM is only a waypoint, its links carry the two hops.
//
// Link load when every TP pair of an 8-GPU node exchanges at once (the TP2 x PP x DP layouts):
// f -> g carries 2/8 of f's message; f -> r carries 1/8 (f's relay part) and r -> g carries 1/8
// (g pulling f's part) + 1/8 (r's own part relayed through g), so every directed link moves 2/8 of
// a message: ~4x the one-link rate (7x for a lone pair). The reference has nothing like it: its TP
// collectives are stock NCCL rings.
//
// Protocol (per call, epoch e identical on both partners; parity = e & 1). e is either a host call
// counter passed by value, or (device epochs, the engine's mode) this rank's device-side call
// counter `epoch` of its signal buffer plus the call's index inside the exchange: the counter is
// advanced by smdt_relay_epoch_bump after the exchange's calls, so a HIP graph that captured an
// exchange replays it with fresh epochs instead of the epochs frozen at capture.
//   send block (part j, sub-block q): wait until the partner freed this (j, q, parity) slot two
//     calls ago (freed >= e - 2), copy its sub-range into host(j)'s slot with sc0|sc1 stores, drain
//     (vmcnt 0), barrier, publish ready[j][q] = e in the PARTNER's signal buffer.
//   recv block (j, q): wait ready[j][q] >= e (own uncached word), read the sub-range from host(j)
//     with sc0|sc1 loads, drain, publish freed[j][q] = e in the SENDER's signal buffer.
// Every directed flow owns its slots on every host (slot index = source rank), so flows never
// share staging. All spins are bounded; on timeout the block sets the sticky error word of its own
// signal buffer and a recv block NaN-fills its output range, so a lost peer can neither hang the
// GPU nor pass silently. Loopback (tests on one GPU): gridDim.y = W virtual ranks in one launch.
#include <stddef.h>

#include "common.h"
#include "launchers.h"
#include "xgmi_sync.h"

namespace smdt {
namespace relay {

using xg::kSysAux;
using xg::load_sys;
using xg::rsrc;
using xg::store_sys;
using xg::u32x4;

constexpr int kMaxRanks = 8;
constexpr int kMaxSub = 16;  // blocks per part and direction
constexpr int kThreads = 512;
constexpr uint32_t kSpinLimit = 1u << 22;

struct SignalBuf {
  uint32_t ready[kMaxRanks][kMaxSub];  // written by my partner's send blocks
  uint32_t freed[kMaxRanks][kMaxSub];  // written by my partner's recv blocks
  uint32_t error;                        // != 0: a spin timed out (sticky)
  uint32_t spin_limit;                   // polls before giving up (0: kSpinLimit); set by the host
  uint32_t epoch;                        // device epochs: calls completed (smdt_relay_epoch_bump)
  uint32_t pad;
};

struct Peers {
  char* stage[kMaxRanks];
  SignalBuf* sig[kMaxRanks];
  int partner[kMaxRanks];
};

struct Args {
  const u32x4* in;
  u32x4* out;
  int64_t in_rank_stride, out_rank_stride;  // loopback rows (vectors)
  int64_t nvec;                             // 16-byte vectors of this call's message
  int64_t part;                             // vectors per part
  int64_t slot;                             // vectors per (flow, parity) slot (>= 2 * part)
  uint32_t epoch;   // host mode: the call's epoch; device mode: its index (>= 1) within the exchange
  int dev_epoch;    // 1: e = own signal buffer's counter + epoch
  int sub;
};

__device__ __forceinline__ bool wait_ge(SignalBuf* me, const uint32_t* f, uint32_t epoch) {
  const uint32_t lim0 = load_sys(&me->spin_limit);
  const uint32_t lim = lim0 != 0u ? lim0 : kSpinLimit;
  for (uint32_t spins = 0;; ++spins) {
    const uint32_t v = load_sys(f);
    if ((int32_t)(v - epoch) >= 0) return true;
    if ((spins & 255u) == 255u && load_sys(&me->error) != 0u) return false;
    if (spins > lim) {
      store_sys(&me->error, 1u);
      return false;
    }
    __builtin_amdgcn_s_sleep(2);
  }
}

// Host GPU of part j of the flow f -> g: parts 0, 1 at g, part 2 + k at the k-th other rank.
template <int W>
__device__ __forceinline__ int host_of(int j, int f, int g) {
  if (j < 2) return g;
  int k = j - 2;
#pragma unroll
  for (int r = 0; r < W; ++r) {
    if (r == f || r == g) continue;
    if (k-- == 0) return r;
  }
  return g;
}

template <typename T, int W>
__global__ __launch_bounds__(kThreads) void relay_kernel(Peers P, int rank0, Args a) {
  __shared__ int s_ok;
  const int rank = rank0 + (int)blockIdx.y;
  const u32x4* __restrict__ in = a.in + (int64_t)blockIdx.y * a.in_rank_stride;
  u32x4* __restrict__ out = a.out + (int64_t)blockIdx.y * a.out_rank_stride;
  const int nsub = a.sub;
  const bool send = (int)blockIdx.x < W * nsub;
  const int idx = send ? (int)blockIdx.x : (int)blockIdx.x - W * nsub;
  const int j = idx / nsub, q = idx - (idx / nsub) * nsub;
  const int partner = P.partner[rank];
  SignalBuf* me = P.sig[rank];
  const int64_t p0 = min((int64_t)j * a.part, a.nvec), p1 = min(p0 + a.part, a.nvec);
  const int64_t chunk = (a.part + nsub - 1) / nsub;
  const int64_t v0 = min(p0 + (int64_t)q * chunk, p1), v1 = min(v0 + chunk, p1);
  const uint32_t e = (a.dev_epoch ? load_sys(&me->epoch) : 0u) + a.epoch;
  const int64_t par = e & 1u;
  if (threadIdx.x == 0) s_ok = load_sys(&me->error) == 0u;
  __syncthreads();

  if (send) {
    if (!s_ok) return;
    if (e > 2u && threadIdx.x == 0 && !wait_ge(me, &me->freed[j][q], e - 2u)) s_ok = 0;
    __syncthreads();
    if (!s_ok) return;
    const int host = host_of<W>(j, rank, partner);
    const int64_t off = ((int64_t)rank * 2 + par) * a.slot + (j < 2 ? (int64_t)j * a.part : 0);
    const auto dst = rsrc(P.stage[host] + off * 16, (uint32_t)(a.part * 16));
    constexpr int U = 4;
    int64_t v = v0 + threadIdx.x;
    for (; v + (U - 1) * kThreads < v1; v += U * kThreads) {
      u32x4 x[U];
#pragma unroll
      for (int u = 0; u < U; ++u) x[u] = in[v + u * kThreads];
#pragma unroll
      for (int u = 0; u < U; ++u)
        __builtin_amdgcn_raw_buffer_store_b128(x[u], dst, (int)((v + u * kThreads - p0) * 16), 0, kSysAux);
    }
    for (; v < v1; v += kThreads) __builtin_amdgcn_raw_buffer_store_b128(in[v], dst, (int)((v - p0) * 16), 0, kSysAux);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) store_sys(&P.sig[partner]->ready[j][q], e);
    return;
  }

  // receive the partner's part j, sub-range q
  const int src = partner;
  auto fail = [&]() {
    const u32x4 nanv = xg::nan16<T>();
    for (int64_t v = v0 + threadIdx.x; v < v1; v += kThreads) out[v] = nanv;
  };
  if (!s_ok) {
    fail();
    return;
  }
  if (threadIdx.x == 0 && !wait_ge(me, &me->ready[j][q], e)) s_ok = 0;
  __syncthreads();
  if (!s_ok) {
    fail();
    return;
  }
  const int host = host_of<W>(j, src, rank);
  const int64_t off = ((int64_t)src * 2 + par) * a.slot + (j < 2 ? (int64_t)j * a.part : 0);
  const auto from = rsrc(P.stage[host] + off * 16, (uint32_t)(a.part * 16));
  constexpr int U = 8;  // remote reads: keep many in flight per thread
  int64_t v = v0 + threadIdx.x;
  for (; v + (U - 1) * kThreads < v1; v += U * kThreads) {
    u32x4 x[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
      x[u] = __builtin_amdgcn_raw_buffer_load_b128(from, (int)((v + u * kThreads - p0) * 16), 0, kSysAux);
#pragma unroll
    for (int u = 0; u < U; ++u) out[v + u * kThreads] = x[u];
  }
  for (; v < v1; v += kThreads) out[v] = __builtin_amdgcn_raw_buffer_load_b128(from, (int)((v - p0) * 16), 0, kSysAux);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) store_sys(&P.sig[src]->freed[j][q], e);
}

// Device epochs: advance the call counter of each local rank's signal buffer by n (the calls of the
// exchange just issued). One vector atomic per rank: never a scalar-memory write.
__global__ void epoch_bump_kernel(Peers P, int rank0, int nlocal, uint32_t n) {
  const int t = (int)threadIdx.x;
  if (t < nlocal) __hip_atomic_fetch_add(&P.sig[rank0 + t]->epoch, n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

template <typename T>
hipError_t launch_t(int world, const Peers& P, int rank0, int nranks_local, const Args& a, hipStream_t st) {
  const dim3 grid(2 * world * a.sub, nranks_local);
  switch (world) {
    case 2: hipLaunchKernelGGL((relay_kernel<T, 2>), grid, dim3(kThreads), 0, st, P, rank0, a); break;
    case 4: hipLaunchKernelGGL((relay_kernel<T, 4>), grid, dim3(kThreads), 0, st, P, rank0, a); break;
    case 8: hipLaunchKernelGGL((relay_kernel<T, 8>), grid, dim3(kThreads), 0, st, P, rank0, a); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace relay
}  // namespace smdt

using namespace smdt;

extern "C" {

int64_t smdt_relay_signal_bytes() { return (int64_t)sizeof(relay::SignalBuf); }
int64_t smdt_relay_word_offset(int which) {
  return which == 0   ? (int64_t)offsetof(relay::SignalBuf, error)
         : which == 1 ? (int64_t)offsetof(relay::SignalBuf, spin_limit)
                      : (int64_t)offsetof(relay::SignalBuf, epoch);
}

// Protocol reset (host, between exchanges, after every rank synchronised): zero this rank's ready /
// freed flags and its device epoch, so the next call is epoch 1 with no slot waits. Used when
// the engine changes its blocks per part (XgmiRelay.tune_sub): the (part, block) -> sub-range map
// changes, so flags of the old map must not satisfy waits of the new one.
hipError_t smdt_relay_reset(void* sig, hipStream_t st) {
  if (!sig) return hipErrorInvalidValue;
  hipError_t e = hipMemsetAsync(sig, 0, offsetof(relay::SignalBuf, error), st);
  if (e != hipSuccess) return e;
  return hipMemsetAsync((char*)sig + offsetof(relay::SignalBuf, epoch), 0, sizeof(uint32_t), st);
}

hipError_t smdt_relay_epoch_bump(void* const* sig_ptrs, int world, int rank, int nranks_local, uint32_t n,
                                 hipStream_t st) {
  if (world < 1 || world > relay::kMaxRanks || rank < 0 || nranks_local < 1 || rank + nranks_local > world)
    return hipErrorInvalidValue;
  relay::Peers P{};
  for (int r = 0; r < world; ++r) {
    if (!sig_ptrs[r]) return hipErrorInvalidValue;
    P.sig[r] = (relay::SignalBuf*)sig_ptrs[r];
  }
  hipLaunchKernelGGL(relay::epoch_bump_kernel, dim3(1), dim3(64), 0, st, P, rank, nranks_local, n);
  return hipGetLastError();
}
int smdt_relay_max_sub() { return relay::kMaxSub; }

hipError_t smdt_relay_read_error(void* sig, int* err) {
  uint32_t v = 0;
  const hipError_t e = hipMemcpy(&v, (char*)sig + offsetof(relay::SignalBuf, error), 4, hipMemcpyDeviceToHost);
  *err = (int)v;
  return e;
}

hipError_t smdt_xgmi_relay(int dtype, const void* in, void* out, int64_t in_rank_stride, int64_t out_rank_stride,
                           int64_t n, void* const* stage_ptrs, void* const* sig_ptrs, const int* partners, int world,
                           int rank, int nranks_local, int64_t slot_bytes, int sub, uint32_t epoch, int dev_epoch,
                           hipStream_t st) {
  if (world != 2 && world != 4 && world != 8) return hipErrorInvalidValue;
  if (rank < 0 || nranks_local < 1 || rank + nranks_local > world || sub < 1 || sub > relay::kMaxSub || epoch == 0)
    return hipErrorInvalidValue;
  const int esz = dtype == 0 ? 4 : 2;
  if (n <= 0 || (n * esz) % 16 != 0 || slot_bytes % 16 != 0 || slot_bytes > (1ll << 31) - 16) return hipErrorInvalidValue;
  if ((((uintptr_t)in | (uintptr_t)out) & 15) != 0 || (in_rank_stride * esz) % 16 != 0 ||
      (out_rank_stride * esz) % 16 != 0)
    return hipErrorInvalidValue;
  relay::Args a;
  a.nvec = n * esz / 16;
  a.part = (a.nvec + world - 1) / world;
  a.slot = slot_bytes / 16;
  if (2 * a.part > a.slot) return hipErrorInvalidValue;  // the host splits larger messages
  relay::Peers P{};
  for (int r = 0; r < world; ++r) {
    if (!stage_ptrs[r] || !sig_ptrs[r]) return hipErrorInvalidValue;
    const int p = partners[r];
    if (p < 0 || p >= world || p == r || partners[p] != r) return hipErrorInvalidValue;
    P.stage[r] = (char*)stage_ptrs[r];
    P.sig[r] = (relay::SignalBuf*)sig_ptrs[r];
    P.partner[r] = p;
  }
  a.in = (const relay::u32x4*)in;
  a.out = (relay::u32x4*)out;
  a.in_rank_stride = in_rank_stride * esz / 16;
  a.out_rank_stride = out_rank_stride * esz / 16;
  a.epoch = epoch;
  a.dev_epoch = dev_epoch ? 1 : 0;
  a.sub = sub;
  switch (dtype) {
    case 0: return relay::launch_t<float>(world, P, rank, nranks_local, a, st);
    case 1: return relay::launch_t<bf16>(world, P, rank, nranks_local, a, st);
    case 2: return relay::launch_t<f16>(world, P, rank, nranks_local, a, st);
    default: return hipErrorInvalidValue;
  }
}

}  // extern "C"
