// Single-node all-reduce over xGMI peer memory (SURVEY C2', C4, §5.8, §7.4 item 1): every rank
// maps every other rank's staging buffer through HIP IPC and reads it directly, so ONE kernel
// drives all 7 xGMI links of an MI355X at once instead of a ring's one link per direction.
//
// Reference context: the reference all-reduces DDP buckets and TP activations through NCCL /
// SMDDP (`1_training_mnist_ddp/pytorch_mnist_ddp.py:87-104`, TP=4 all-reduces of 18.9 MB per
// layer in NB3) and has no custom all-reduce; nothing here is modelled on code.
//
// Algorithms (chosen per call by the host):
//   one-shot       : stage my input into my region A, signal every peer, wait for every peer,
//                    then reduce the WHOLE tensor by reading all W staging regions (latency-optimal).
//   two-shot       : same staging + barrier, then rank r reduces only slice r of each block's range
//                    (a reduce-scatter through peer reads), publishes it in region B, a second
//                    barrier, and every rank gathers the W-1 other slices (each link carries 2/W of
//                    the message).
//   reduce-scatter : input = W slices of ns vectors (slice d at in + d * slice stride); block b
//                    stages sub-range b of EVERY slice, one barrier, then reduces sub-range b of
//                    slice `rank` over the W staged copies (ZeRO gradient shards; each link carries
//                    1/W of the message).
//   all-gather     : input = ns vectors; block b stages its sub-range, one barrier, then copies
//                    sub-range b of every peer's staged slice into out slice r (ZeRO parameters).
// Reductions accumulate in fp32 in rank order 0..W-1, so every rank ends with bit-identical results
// (TP replicas must stay identical). A block's staging and reading ranges coincide, so the
// per-block barrier is all the ordering a call needs, and an output that aliases the input (ZeRO's
// in-place reduce-scatter into the bucket, in-place all-gather) is safe: a block overwrites only
// bytes it staged itself before its barrier.
//
// Cross-device visibility (MI355X_MICROARCH.md "visibility", system scope because the consumer is
// another GPU): every staged byte is stored with sc0|sc1 (write-through) buffer stores, every wave
// drains with s_waitcnt vmcnt(0), the block joins a barrier, and ONE lane per peer then stores the
// epoch flag into that peer's signal buffer with a system-scope atomic store. Consumers poll their
// own (uncached) signal words with system-scope relaxed loads and read peer data ONLY with sc0|sc1
// buffer loads, which bypass both cache levels: no stale line can be hit.
//
// Reuse without an end barrier: staging is double-buffered on the parity of a per-block call
// counter kept in device memory (hipGraph-replayable, no host-side epoch). The grid size is a
// fixed property of an engine, so every block index takes part in every call and all counters
// (hence all parities) advance together. A rank can be at most one call ahead of any peer (its
// next barrier needs that peer's flag, which the peer only sets after finishing the previous
// call in stream order), so it only ever overwrites the half a slower peer has finished reading.
// Flags are compared with ">=" on monotonically increasing epochs for the same reason.
//
// Every spin is bounded: on timeout the block records a sticky error word in its own signal
// buffer, fills its output range with NaN and exits, so a missing peer can never hang the GPU and
// a failed reduction cannot pass silently (the host can also read the word back).
//
// Loopback mode (tests on ONE GPU): gridDim.y = W virtual ranks in ONE launch, rank = blockIdx.y,
// in/out strided by `io_stride` per rank; the host keeps W x blocks small enough that every
// workgroup is co-resident, so the barriers between them make progress.
#include <stddef.h>

#include "common.h"
#include "launchers.h"
#include "xgmi_sync.h"

namespace smdt {
namespace ar {

constexpr int kMaxRanks = 8;
constexpr int kMaxBlocks = 256;
constexpr int kThreads = 512;
constexpr uint32_t kSpinLimit = 1u << 22;  // polls of an uncached word (~1 us each): seconds

struct SignalBuf {
  uint32_t flag[kMaxBlocks][kMaxRanks];  // flag[b][src]: written remotely by rank src's block b
  uint32_t counter[kMaxBlocks];          // this rank's call counter per block (local only)
  uint32_t error;                        // != 0: a spin timed out (sticky)
  uint32_t spin_limit;                   // polls before giving up (0: kSpinLimit); set by the host
  uint32_t pad[2];
};

struct Peers {
  char* data[kMaxRanks];      // staging buffers: 4 regions of region_bytes (2 halves x {A, B})
  SignalBuf* sig[kMaxRanks];  // signal buffers
};

using xg::load_sys;
using xg::rsrc;
using xg::store_sys;
using xg::u32x4;

// Poll my own flag word until it reaches `epoch`; give up when the sticky error is set or the
// spin limit runs out (then set the error). Returns false on failure.
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

// Barrier among block b of every rank: publish `epoch` to every peer, then wait for every peer's
// epoch. Each wave drains its own staging stores (vmcnt(0)) before the workgroup barrier that
// orders all of them ahead of the flag stores.
template <int W>
__device__ __forceinline__ bool block_barrier(const Peers& P, int rank, int b, uint32_t epoch, int* s_ok) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const int t = threadIdx.x;
  if (t < W) {
    store_sys(&P.sig[t]->flag[b][rank], epoch);
    if (!wait_ge(P.sig[rank], &P.sig[rank]->flag[b][t], epoch)) *s_ok = 0;
  }
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // no instruction: keeps loads below
  return *s_ok != 0;
}

using xg::kSysAux;

template <typename T> constexpr int E16 = 16 / (int)sizeof(T);

template <typename T>
__device__ __forceinline__ void acc16(float (&a)[E16<T>], u32x4 raw) {
  if constexpr (sizeof(T) == 4) {
    const f32x4 v = __builtin_bit_cast(f32x4, raw);
#pragma unroll
    for (int j = 0; j < 4; ++j) a[j] += v[j];
  } else {
    const u16x8 v = __builtin_bit_cast(u16x8, raw);
#pragma unroll
    for (int j = 0; j < E16<T>; ++j) {
      const unsigned short bits = v[j];
      T x;
      __builtin_memcpy(&x, &bits, 2);
      a[j] += to_f32(x);
    }
  }
}

template <typename T>
__device__ __forceinline__ u32x4 pack16(const float (&a)[E16<T>], float scale) {
  if constexpr (sizeof(T) == 4) {
    f32x4 r;
#pragma unroll
    for (int j = 0; j < 4; ++j) r[j] = a[j] * scale;
    return __builtin_bit_cast(u32x4, r);
  } else {
    u16x8 v;
#pragma unroll
    for (int j = 0; j < E16<T>; ++j) {
      const T x = from_f32<T>(a[j] * scale);
      unsigned short bits;
      __builtin_memcpy(&bits, &x, 2);
      v[j] = bits;
    }
    return __builtin_bit_cast(u32x4, v);
  }
}

template <typename T>
__device__ __forceinline__ void nan_fill(u32x4* __restrict__ out, int64_t v0, int64_t v1) {
  const u32x4 q = xg::nan16<T>();
  for (int64_t v = v0 + threadIdx.x; v < v1; v += kThreads) out[v] = q;
}

// out[v] = scale * sum_r region(r)[v] for v in [v0, v1), summed in rank order. kPublish also
// stages the result (sc0|sc1) into my region B for the two-shot gather.
template <typename T, int W, bool kPublish>
__device__ __forceinline__ void reduce_range(const Peers& P, int64_t reg_off, uint32_t reg_bytes, int64_t v0,
                                             int64_t v1, float scale, u32x4* __restrict__ out,
                                             __amdgpu_buffer_rsrc_t pub) {
  __amdgpu_buffer_rsrc_t src[W];
#pragma unroll
  for (int r = 0; r < W; ++r) src[r] = rsrc(P.data[r] + reg_off, reg_bytes);
  for (int64_t v = v0 + threadIdx.x; v < v1; v += kThreads) {
    u32x4 raw[W];
#pragma unroll
    for (int r = 0; r < W; ++r) raw[r] = __builtin_amdgcn_raw_buffer_load_b128(src[r], (int)(v * 16), 0, kSysAux);
    float a[E16<T>];
#pragma unroll
    for (int j = 0; j < E16<T>; ++j) a[j] = 0.f;
#pragma unroll
    for (int r = 0; r < W; ++r) acc16<T>(a, raw[r]);
    const u32x4 o = pack16<T>(a, scale);
    out[v] = o;
    if constexpr (kPublish) __builtin_amdgcn_raw_buffer_store_b128(o, pub, (int)(v * 16), 0, kSysAux);
  }
}

enum Mode { kOneShot = 0, kTwoShot = 1, kReduceScatter = 2, kAllGather = 3 };

// Call arguments (by value). Vector (16-byte) units throughout. Loopback: blockIdx.y = virtual
// rank, whose in / out start in_rank_stride / out_rank_stride vectors after the previous one's.
struct Args {
  const u32x4* in;
  u32x4* out;
  int64_t in_rank_stride, out_rank_stride;
  int64_t nvec;          // all-reduce: vectors of the tensor; RS / AG: vectors per slice
  int64_t slice_stride;  // RS: between input slices; AG: between output slices
  int64_t chunk;         // vectors per block (per slice for RS / AG)
  int64_t region_bytes;
  float scale;
};

template <typename T, int W, int MODE>
__global__ __launch_bounds__(kThreads) void collective_kernel(Peers P, int rank0, Args a) {
  __shared__ uint32_t s_counter;
  __shared__ int s_ok;
  const int b = blockIdx.x;
  const int rank = rank0 + (int)blockIdx.y;
  const u32x4* __restrict__ in = a.in + (int64_t)blockIdx.y * a.in_rank_stride;
  u32x4* __restrict__ out = a.out + (int64_t)blockIdx.y * a.out_rank_stride;
  SignalBuf* me = P.sig[rank];
  const int64_t nvec = a.nvec, chunk = a.chunk;
  const int64_t v0 = (int64_t)b * chunk < nvec ? (int64_t)b * chunk : nvec;
  const int64_t v1 = v0 + chunk < nvec ? v0 + chunk : nvec;
  // ranges this block writes (NaN-filled on failure)
  auto fail = [&]() {
    if constexpr (MODE == kReduceScatter) {
      nan_fill<T>(out, v0, v1);
    } else if constexpr (MODE == kAllGather) {
      for (int r = 0; r < W; ++r) nan_fill<T>(out + (int64_t)r * a.slice_stride, v0, v1);
    } else {
      nan_fill<T>(out, v0, v1);
    }
  };
  if (threadIdx.x == 0) {
    s_counter = load_sys(&me->counter[b]);
    s_ok = load_sys(&me->error) == 0u;
  }
  __syncthreads();
  if (!s_ok) {  // a previous call failed: never wait on peers again (the host must rebuild)
    fail();
    return;
  }
  const uint32_t c = s_counter;
  const uint32_t half = (c >> 1) & 1u;
  const uint32_t rb = (uint32_t)a.region_bytes;
  const int64_t offA = (int64_t)(2 * half) * a.region_bytes;
  const int64_t offB = offA + a.region_bytes;

  {  // 1) stage my input, write-through, so peers read it from memory
    const auto mine = rsrc(P.data[rank] + offA, rb);
    if constexpr (MODE == kReduceScatter) {
#pragma unroll
      for (int d = 0; d < W; ++d) {
        const u32x4* src = in + (int64_t)d * a.slice_stride;
        const int64_t base = (int64_t)d * nvec;
        for (int64_t v = v0 + threadIdx.x; v < v1; v += kThreads)
          __builtin_amdgcn_raw_buffer_store_b128(src[v], mine, (int)((base + v) * 16), 0, kSysAux);
      }
    } else {
      for (int64_t v = v0 + threadIdx.x; v < v1; v += kThreads)
        __builtin_amdgcn_raw_buffer_store_b128(in[v], mine, (int)(v * 16), 0, kSysAux);
    }
  }
  if (!block_barrier<W>(P, rank, b, c + 1, &s_ok)) {
    fail();
    return;
  }

  if constexpr (MODE == kOneShot) {
    reduce_range<T, W, false>(P, offA, rb, v0, v1, a.scale, out, rsrc(nullptr, 0));
  } else if constexpr (MODE == kReduceScatter) {
    // 2) my slice's sub-range, summed over the W staged copies (rank order)
    u32x4* o = out - (int64_t)rank * nvec;  // reduce_range indexes by the staged position
    reduce_range<T, W, false>(P, offA, rb, (int64_t)rank * nvec + v0, (int64_t)rank * nvec + v1, a.scale, o,
                              rsrc(nullptr, 0));
  } else if constexpr (MODE == kAllGather) {
    // 2) every rank's sub-range (mine from my own input)
#pragma unroll
    for (int r = 0; r < W; ++r) {
      u32x4* o = out + (int64_t)r * a.slice_stride;
      if (r == rank) {
        if (in != o)
          for (int64_t v = v0 + threadIdx.x; v < v1; v += kThreads) o[v] = in[v];
        continue;
      }
      const auto src = rsrc(P.data[r] + offA, rb);
      for (int64_t v = v0 + threadIdx.x; v < v1; v += kThreads)
        o[v] = __builtin_amdgcn_raw_buffer_load_b128(src, (int)(v * 16), 0, kSysAux);
    }
  } else {
    // 2) reduce-scatter: I own slice `rank` of this block's range; publish it in my region B
    const int64_t sl = (v1 - v0 + W - 1) / W;
    auto lo = [&](int r) { const int64_t x = v0 + (int64_t)r * sl; return x < v1 ? x : v1; };
    auto hi = [&](int r) { const int64_t x = lo(r) + sl; return x < v1 ? x : v1; };
    reduce_range<T, W, true>(P, offA, rb, lo(rank), hi(rank), a.scale, out, rsrc(P.data[rank] + offB, rb));
    if (!block_barrier<W>(P, rank, b, c + 2, &s_ok)) {
      fail();
      return;
    }
    // 3) all-gather the other ranks' slices from their region B
#pragma unroll
    for (int r = 0; r < W; ++r) {
      if (r == rank) continue;
      const auto src = rsrc(P.data[r] + offB, rb);
      const int64_t g1 = hi(r);
      for (int64_t v = lo(r) + threadIdx.x; v < g1; v += kThreads)
        out[v] = __builtin_amdgcn_raw_buffer_load_b128(src, (int)(v * 16), 0, kSysAux);
    }
  }
  if (threadIdx.x == 0) store_sys(&me->counter[b], c + 2);
}

template <typename T, int W>
hipError_t launch_w(int mode, const Peers& P, int rank0, int nranks_local, const Args& a, int blocks, hipStream_t st) {
  const dim3 grid(blocks, nranks_local);  // ALL blocks, also those whose range is empty
  switch (mode) {
    case kOneShot: hipLaunchKernelGGL((collective_kernel<T, W, kOneShot>), grid, dim3(kThreads), 0, st, P, rank0, a); break;
    case kTwoShot: hipLaunchKernelGGL((collective_kernel<T, W, kTwoShot>), grid, dim3(kThreads), 0, st, P, rank0, a); break;
    case kReduceScatter: hipLaunchKernelGGL((collective_kernel<T, W, kReduceScatter>), grid, dim3(kThreads), 0, st, P, rank0, a); break;
    case kAllGather: hipLaunchKernelGGL((collective_kernel<T, W, kAllGather>), grid, dim3(kThreads), 0, st, P, rank0, a); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

template <typename T>
hipError_t launch_t(int mode, const Peers& P, int world, int rank0, int nranks_local, const Args& a, int blocks,
                    hipStream_t st) {
  switch (world) {
    case 2: return launch_w<T, 2>(mode, P, rank0, nranks_local, a, blocks, st);
    case 4: return launch_w<T, 4>(mode, P, rank0, nranks_local, a, blocks, st);
    case 8: return launch_w<T, 8>(mode, P, rank0, nranks_local, a, blocks, st);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace ar
}  // namespace smdt

using namespace smdt;

extern "C" {

int smdt_ar_max_ranks() { return ar::kMaxRanks; }
int smdt_ar_max_blocks() { return ar::kMaxBlocks; }
int64_t smdt_ar_signal_bytes() { return (int64_t)sizeof(ar::SignalBuf); }
// byte offset of a host-visible word of the signal buffer: 0 = sticky error, 1 = spin limit
int64_t smdt_ar_word_offset(int which) {
  return which == 0 ? (int64_t)offsetof(ar::SignalBuf, error) : (int64_t)offsetof(ar::SignalBuf, spin_limit);
}
int smdt_ipc_handle_bytes() { return (int)sizeof(hipIpcMemHandle_t); }

hipError_t smdt_ipc_malloc(int64_t bytes, int uncached, void** ptr) {
  hipError_t e = uncached ? hipExtMallocWithFlags(ptr, (size_t)bytes, hipDeviceMallocUncached)
                          : hipMalloc(ptr, (size_t)bytes);
  if (e != hipSuccess) return e;
  e = hipMemset(*ptr, 0, (size_t)bytes);
  if (e != hipSuccess) return e;
  return hipDeviceSynchronize();
}

hipError_t smdt_ipc_free(void* ptr) { return hipFree(ptr); }

hipError_t smdt_ipc_get_handle(void* ptr, void* handle_out) {
  hipIpcMemHandle_t h;
  const hipError_t e = hipIpcGetMemHandle(&h, ptr);
  if (e == hipSuccess) __builtin_memcpy(handle_out, &h, sizeof(h));
  return e;
}

hipError_t smdt_ipc_open(const void* handle, void** ptr) {
  hipIpcMemHandle_t h;
  __builtin_memcpy(&h, handle, sizeof(h));
  return hipIpcOpenMemHandle(ptr, h, hipIpcMemLazyEnablePeerAccess);
}

hipError_t smdt_ipc_close(void* ptr) { return hipIpcCloseMemHandle(ptr); }

// Sticky error word of one signal buffer (0 = fine). Synchronous device -> host copy.
hipError_t smdt_ar_read_error(void* sig, int* err) {
  uint32_t v = 0;
  const hipError_t e = hipMemcpy(&v, (char*)sig + offsetof(ar::SignalBuf, error), 4, hipMemcpyDeviceToHost);
  *err = (int)v;
  return e;
}

// mode: 0 one-shot / 1 two-shot all-reduce (n = elements of the tensor), 2 reduce-scatter (n =
// elements per slice; input slices slice_stride elements apart, output n elements), 3 all-gather
// (n = elements per slice; output slices slice_stride elements apart). io strides: loopback only.
hipError_t smdt_xgmi_collective(int mode, int dtype, const void* in, void* out, int64_t in_rank_stride,
                                int64_t out_rank_stride, int64_t n, int64_t slice_stride, float scale,
                                void* const* data_ptrs, void* const* sig_ptrs, int world, int rank, int nranks_local,
                                int64_t region_bytes, int blocks, hipStream_t st) {
  if (mode < 0 || mode > 3) return hipErrorInvalidValue;
  if (world < 2 || world > ar::kMaxRanks || rank < 0 || nranks_local < 1 || rank + nranks_local > world)
    return hipErrorInvalidValue;
  if (blocks < 1 || blocks > ar::kMaxBlocks) return hipErrorInvalidValue;
  const int esz = dtype == 0 ? 4 : 2;
  const int64_t staged = mode == 2 ? n * world : n;  // elements one rank stages
  if (n <= 0 || (n * esz) % 16 != 0 || staged * esz > region_bytes || region_bytes > (1ll << 31) - 16 ||
      region_bytes % 16 != 0)
    return hipErrorInvalidValue;
  if (mode >= 2 && (slice_stride < n || (slice_stride * esz) % 16 != 0)) return hipErrorInvalidValue;
  if ((((uintptr_t)in | (uintptr_t)out) & 15) != 0 || (in_rank_stride * esz) % 16 != 0 ||
      (out_rank_stride * esz) % 16 != 0)
    return hipErrorInvalidValue;
  ar::Peers P{};
  for (int r = 0; r < world; ++r) {
    if (!data_ptrs[r] || !sig_ptrs[r]) return hipErrorInvalidValue;
    P.data[r] = (char*)data_ptrs[r];
    P.sig[r] = (ar::SignalBuf*)sig_ptrs[r];
  }
  ar::Args a;
  a.in = (const ar::u32x4*)in;
  a.out = (ar::u32x4*)out;
  a.in_rank_stride = in_rank_stride * esz / 16;
  a.out_rank_stride = out_rank_stride * esz / 16;
  a.nvec = n * esz / 16;
  a.slice_stride = mode >= 2 ? slice_stride * esz / 16 : 0;
  a.chunk = (a.nvec + blocks - 1) / blocks;
  a.region_bytes = region_bytes;
  a.scale = scale;
  switch (dtype) {
    case 0: return ar::launch_t<float>(mode, P, world, rank, nranks_local, a, blocks, st);
    case 1: return ar::launch_t<bf16>(mode, P, world, rank, nranks_local, a, blocks, st);
    case 2: return ar::launch_t<f16>(mode, P, world, rank, nranks_local, a, blocks, st);
    default: return hipErrorInvalidValue;
  }
}

hipError_t smdt_xgmi_allreduce(int dtype, const void* in, void* out, int64_t io_stride, int64_t n, float scale,
                               void* const* data_ptrs, void* const* sig_ptrs, int world, int rank,
                               int nranks_local, int64_t region_bytes, int two_shot, int blocks,
                               hipStream_t st) {
  return smdt_xgmi_collective(two_shot ? 1 : 0, dtype, in, out, io_stride, io_stride, n, 0, scale, data_ptrs,
                              sig_ptrs, world, rank, nranks_local, region_bytes, blocks, st);
}

}  // extern "C"
