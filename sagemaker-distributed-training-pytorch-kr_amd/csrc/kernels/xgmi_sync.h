// Cross-GPU visibility helpers shared by the xGMI collectives (xgmi_allreduce.hip, xgmi_relay.hip).
//
// Producers store peer-visible data with sc0|sc1 (write-through to the owning GPU's HBM), drain
// with s_waitcnt vmcnt(0) and only then publish a flag with a system-scope store; consumers poll
// uncached flag words with system-scope loads and read the data with sc0|sc1 loads, which bypass
// both cache levels (MI355X_MICROARCH.md "visibility": the consumer is another device).
#pragma once

#include "common.h"

namespace smdt {
namespace xg {

using gu32 = __attribute__((address_space(1))) uint32_t;
using u32x4 = __attribute__((ext_vector_type(4))) unsigned;

constexpr int kSysAux = 1 | 16;  // sc0 | sc1: system coherent, bypasses L1 and L2

__device__ __forceinline__ void store_sys(uint32_t* p, uint32_t v) {
  __hip_atomic_store((gu32*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);  // global, never flat
}
__device__ __forceinline__ uint32_t load_sys(const uint32_t* p) {
  return __hip_atomic_load((gu32*)const_cast<uint32_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}

// One 16-byte NaN pattern per element type (fp32 / 2 x bf16 / 2 x fp16 quiet NaNs).
template <typename T>
__device__ __forceinline__ u32x4 nan16() {
  uint32_t w = 0x7fc00000u;
  if constexpr (std::is_same<T, bf16>::value) w = 0x7fc07fc0u;
  if constexpr (std::is_same<T, f16>::value) w = 0x7e007e00u;
  return u32x4{w, w, w, w};
}

}  // namespace xg
}  // namespace smdt
