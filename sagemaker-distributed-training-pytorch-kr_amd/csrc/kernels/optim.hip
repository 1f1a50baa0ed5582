// Fused optimizer kernels for gfx950: Adam/AdamW over flat fp32 master buffers, global grad
// L2-norm + inf/nan detection, scale, and fp32 -> bf16/fp16 parameter copy-out.
//
// Replaces apex `amp_C.multi_tensor_adam` / `multi_tensor_l2norm` / `multi_tensor_scale` and
// DeepSpeed FusedAdam (Megatron `--optimizer adam`, `--clip-grad`,
// /root/reference/3_training_megatron-lm/megatron/arguments.py:700-710, :831-833; DeepSpeed
// `DS_BUILD_FUSED_ADAM=1`, /root/reference/4_training_alpaca_deepspeed/docker/Dockerfile:16-25).
//
// MI355X-first layout: the framework keeps every parameter, gradient and optimizer state in
// ONE contiguous flat buffer per dtype (the grad buffer doubles as the DDP/ZeRO communication
// buffer), so there is no multi-tensor pointer table: an update is a single grid-stride stream
// over 16-byte vectors, bound only by HBM. Every scalar that depends on the step (grad-clip
// coefficient, loss-scale inverse, found-inf flag) is read from device memory, so a whole
// optimizer step runs without a host synchronisation.
#include "common.h"
#include "launchers.h"

namespace smdt {

struct AdamArgs {
  float* master;          // fp32 master weights [n]
  const float* grad;      // fp32 grads [n]
  float* exp_avg;         // [n]
  float* exp_avg_sq;      // [n]
  void* model_out;        // low-precision model copy [n] (optional)
  int model_dtype;        // 1 = bf16, 2 = f16, 0 = none
  int64_t n;
  float lr, beta1, beta2, eps, weight_decay;
  float bc1, bc2;         // bias corrections 1 - beta^t
  int adamw;              // 1: decoupled weight decay; 0: L2 added to grad
  const float* grad_mul;  // device scalar multiplier applied to grads (clip * 1/loss_scale); may be null
  const int* found_inf;   // device flag; when nonzero the step is skipped; may be null
  const float* hyper;     // capturable form: device [lr, bc1, bc2] read at run time (HIP-graph
                          // replays see the current step / lr); null: the scalars above
};


// Stage 1 of the global L2 norm: per-block sum of squares (fp32 or 16-bit input) and an
// inf/nan flag. Stage 2 (`l2norm_finalize_kernel`) sums the block partials in a fixed order.
template <typename T>
__global__ __launch_bounds__(256) void sumsq_kernel(const T* __restrict__ x, int64_t n,
                                                    float* __restrict__ partial,
                                                    int* __restrict__ found_inf) {
  __shared__ float scratch[4];
  constexpr int V = 16 / sizeof(T);
  const int64_t nvec = n / V;
  float acc = 0.f;
  bool bad = false;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < nvec;
       i += (int64_t)gridDim.x * 256) {
    float v[V];
    load_vec<T, V>(x + i * V, v);
#pragma unroll
    for (int j = 0; j < V; ++j) {
      acc += v[j] * v[j];
      bad |= !isfinite(v[j]);
    }
  }
  if (blockIdx.x == 0 && threadIdx.x < (n % V)) {
    float v = to_f32(x[nvec * V + threadIdx.x]);
    acc += v * v;
    bad |= !isfinite(v);
  }
  float s = block_sum(acc, scratch, 4);
  if (threadIdx.x == 0) partial[blockIdx.x] = s;
  if (bad && found_inf) atomicOr(found_inf, 1);
}

// out[0] = sum of the block partials (fixed order: deterministic). The caller may all-reduce
// out[0] across ranks before `clip_coef_kernel` turns it into the grad multiplier.
__global__ void l2norm_finalize_kernel(const float* __restrict__ partial, int nblocks,
                                       float* __restrict__ out) {
  __shared__ float scratch[4];
  float acc = 0.f;
  for (int i = threadIdx.x; i < nblocks; i += 256) acc += partial[i];
  float s = block_sum(acc, scratch, 4);
  if (threadIdx.x == 0) out[0] = s;
}

__global__ void clip_coef_kernel(const float* __restrict__ sumsq, float max_norm, float inv_scale,
                                 float* __restrict__ mul_out, float* __restrict__ norm_out) {
  if (threadIdx.x != 0) return;
  // The grads are still multiplied by the loss scale: un-scale the norm first.
  float norm = sqrtf(*sumsq) * inv_scale;
  if (norm_out) *norm_out = norm;
  float coef = 1.f;
  if (max_norm > 0.f) {
    coef = max_norm / (norm + 1e-6f);
    coef = coef < 1.f ? coef : 1.f;
  }
  *mul_out = coef * inv_scale;
}

template <typename T>
__global__ __launch_bounds__(256) void scale_kernel(T* __restrict__ x, int64_t n,
                                                    const float* __restrict__ mul, float cmul) {
  const float m = mul ? *mul * cmul : cmul;
  constexpr int V = 16 / sizeof(T);
  const int64_t nvec = n / V;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < nvec;
       i += (int64_t)gridDim.x * 256) {
    float v[V];
    load_vec<T, V>(x + i * V, v);
#pragma unroll
    for (int j = 0; j < V; ++j) v[j] *= m;
    store_vec<T, V>(x + i * V, v);
  }
  if (blockIdx.x == 0 && threadIdx.x < (n % V)) {
    int64_t k = nvec * V + threadIdx.x;
    x[k] = from_f32<T>(to_f32(x[k]) * m);
  }
}

// Cast-copy between flat buffers (fp32 master -> bf16 model, or bf16 grads -> fp32 main grads
// with optional accumulate).
template <typename TI, typename TO>
__global__ __launch_bounds__(256) void cast_kernel(const TI* __restrict__ x, TO* __restrict__ y,
                                                   int64_t n, int accumulate) {
  constexpr int V = 8;
  const int64_t nvec = n / V;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < nvec;
       i += (int64_t)gridDim.x * 256) {
    float v[V];
    load_vec<TI, V>(x + i * V, v);
    if (accumulate) {
      float o[V];
      load_vec<TO, V>(y + i * V, o);
#pragma unroll
      for (int j = 0; j < V; ++j) v[j] += o[j];
    }
    store_vec<TO, V>(y + i * V, v);
  }
  if (blockIdx.x == 0 && threadIdx.x < (n % V)) {
    int64_t k = nvec * V + threadIdx.x;
    float v = to_f32(x[k]);
    if (accumulate) v += to_f32(y[k]);
    y[k] = from_f32<TO>(v);
  }
}

// Fused Adam / AdamW, one batch per thread: thread t of block b updates the U float4 vectors
// b*256*U + u*256 + t (u < U; coalesced per u) of every state stream, all loads in flight at
// once, no grid-stride loop; the grid covers the whole buffer. On the GPT-2 345M buffer (355 M
// params: fp32 master / grad / m / v + bf16 copy) U = 1 runs at 5.7 TB/s (1.87 ms) against
// 4.5 TB/s (2.37 ms) for the former grid-stride form capped at 2048 blocks; U = 2 / 4: 5.5-5.6
// (benchmarks/bench_adam.py, profiles/r4_adam_batch/).
template <typename TO, int U>
__global__ __launch_bounds__(256) void adam_batch_kernel(AdamArgs a) {
  if (a.found_inf && *a.found_inf) return;
  const float gm = a.grad_mul ? *a.grad_mul : 1.f;
  const int64_t nvec = a.n / 4;
  const float lr = a.hyper ? a.hyper[0] : a.lr;
  const float step_size = lr / (a.hyper ? a.hyper[1] : a.bc1);
  const float rbc2 = rsqrtf(a.hyper ? a.hyper[2] : a.bc2);
  const int64_t base = (int64_t)blockIdx.x * 256 * U + threadIdx.x;
  f32x4 p[U], g[U], m[U], v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t i = base + u * 256;
    if (i < nvec) {
      p[u] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(a.master) + i);
      g[u] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(a.grad) + i);
      m[u] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(a.exp_avg) + i);
      v[u] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(a.exp_avg_sq) + i);
    }
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t i = base + u * 256;
    if (i >= nvec) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float gj = g[u][j] * gm;
      if (!a.adamw) gj += a.weight_decay * p[u][j];
      m[u][j] = a.beta1 * m[u][j] + (1.f - a.beta1) * gj;
      v[u][j] = a.beta2 * v[u][j] + (1.f - a.beta2) * gj * gj;
      float denom = sqrtf(v[u][j]) * rbc2 + a.eps;
      float upd = m[u][j] / denom;
      if (a.adamw) p[u][j] -= lr * a.weight_decay * p[u][j];
      p[u][j] -= step_size * upd;
    }
    __builtin_nontemporal_store(p[u], reinterpret_cast<f32x4*>(a.master) + i);
    __builtin_nontemporal_store(m[u], reinterpret_cast<f32x4*>(a.exp_avg) + i);
    __builtin_nontemporal_store(v[u], reinterpret_cast<f32x4*>(a.exp_avg_sq) + i);
    if constexpr (!std::is_same<TO, float>::value) {
      if (a.model_out) {
        TO* o = reinterpret_cast<TO*>(a.model_out) + i * 4;
        using v4 = __attribute__((ext_vector_type(4))) unsigned short;
        v4 w;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          TO t = (TO)p[u][j];
          unsigned short bits;
          __builtin_memcpy(&bits, &t, 2);
          w[j] = bits;
        }
        __builtin_nontemporal_store(w, reinterpret_cast<v4*>(o));
      }
    }
  }
  if (blockIdx.x == 0 && threadIdx.x < (a.n & 3)) {   // scalar tail (n not a multiple of 4)
    int64_t k = nvec * 4 + threadIdx.x;
    float pp = a.master[k], gj = a.grad[k] * gm, mm = a.exp_avg[k], vv = a.exp_avg_sq[k];
    if (!a.adamw) gj += a.weight_decay * pp;
    mm = a.beta1 * mm + (1.f - a.beta1) * gj;
    vv = a.beta2 * vv + (1.f - a.beta2) * gj * gj;
    float denom = sqrtf(vv) * rbc2 + a.eps;
    if (a.adamw) pp -= lr * a.weight_decay * pp;
    pp -= step_size * (mm / denom);
    a.master[k] = pp;
    a.exp_avg[k] = mm;
    a.exp_avg_sq[k] = vv;
    if constexpr (!std::is_same<TO, float>::value) {
      if (a.model_out) reinterpret_cast<TO*>(a.model_out)[k] = (TO)pp;
    }
  }
}

}  // namespace smdt

using namespace smdt;

extern "C" hipError_t smdt_adam(float* master, const float* grad, float* m, float* v,
                                void* model_out, int model_dtype, int64_t n, float lr,
                                float beta1, float beta2, float eps, float wd, float bc1,
                                float bc2, int adamw, const float* grad_mul,
                                const int* found_inf, const float* hyper, hipStream_t st) {
  AdamArgs a{master, grad, m, v, model_out, model_dtype, n, lr, beta1, beta2, eps, wd, bc1, bc2,
             adamw, grad_mul, found_inf, hyper};
  const int64_t blocks = (n / 4 + 255) / 256;
  if (blocks > 0x7FFFFFFF) return hipErrorInvalidValue;
  const dim3 gb((unsigned)(blocks > 0 ? blocks : 1));
  if (model_dtype == 1) hipLaunchKernelGGL((adam_batch_kernel<bf16, 1>), gb, dim3(256), 0, st, a);
  else if (model_dtype == 2) hipLaunchKernelGGL((adam_batch_kernel<f16, 1>), gb, dim3(256), 0, st, a);
  else hipLaunchKernelGGL((adam_batch_kernel<float, 1>), gb, dim3(256), 0, st, a);
  return hipGetLastError();
}

extern "C" int smdt_sumsq_nblocks(int64_t n) { return stream_grid(n / 4 + 1, 256 * 4); }

extern "C" hipError_t smdt_sumsq(int dtype, const void* x, int64_t n, float* partial, int nblocks,
                                 float* out, int* found_inf, hipStream_t st) {
  if (dtype == 1) hipLaunchKernelGGL(sumsq_kernel<bf16>, dim3(nblocks), dim3(256), 0, st, (const bf16*)x, n, partial, found_inf);
  else if (dtype == 2) hipLaunchKernelGGL(sumsq_kernel<f16>, dim3(nblocks), dim3(256), 0, st, (const f16*)x, n, partial, found_inf);
  else hipLaunchKernelGGL(sumsq_kernel<float>, dim3(nblocks), dim3(256), 0, st, (const float*)x, n, partial, found_inf);
  hipLaunchKernelGGL(l2norm_finalize_kernel, dim3(1), dim3(256), 0, st, partial, nblocks, out);
  return hipGetLastError();
}

extern "C" hipError_t smdt_clip_coef(const float* sumsq, float max_norm, float inv_scale,
                                     float* mul_out, float* norm_out, hipStream_t st) {
  hipLaunchKernelGGL(clip_coef_kernel, dim3(1), dim3(64), 0, st, sumsq, max_norm, inv_scale,
                     mul_out, norm_out);
  return hipGetLastError();
}

extern "C" hipError_t smdt_scale(int dtype, void* x, int64_t n, const float* mul, float cmul,
                                 hipStream_t st) {
  int grid = stream_grid(n / 8 + 1, 256);
  if (dtype == 1) hipLaunchKernelGGL(scale_kernel<bf16>, dim3(grid), dim3(256), 0, st, (bf16*)x, n, mul, cmul);
  else if (dtype == 2) hipLaunchKernelGGL(scale_kernel<f16>, dim3(grid), dim3(256), 0, st, (f16*)x, n, mul, cmul);
  else hipLaunchKernelGGL(scale_kernel<float>, dim3(grid), dim3(256), 0, st, (float*)x, n, mul, cmul);
  return hipGetLastError();
}

extern "C" hipError_t smdt_cast(int in_dtype, int out_dtype, const void* x, void* y, int64_t n,
                                int accumulate, hipStream_t st) {
  int grid = stream_grid(n / 8 + 1, 256);
#define SMDT_CAST(TI, TO) hipLaunchKernelGGL((cast_kernel<TI, TO>), dim3(grid), dim3(256), 0, st, (const TI*)x, (TO*)y, n, accumulate)
  if (in_dtype == 0 && out_dtype == 1) SMDT_CAST(float, bf16);
  else if (in_dtype == 0 && out_dtype == 2) SMDT_CAST(float, f16);
  else if (in_dtype == 1 && out_dtype == 0) SMDT_CAST(bf16, float);
  else if (in_dtype == 2 && out_dtype == 0) SMDT_CAST(f16, float);
  else if (in_dtype == 0 && out_dtype == 0) SMDT_CAST(float, float);
  else return hipErrorInvalidValue;
#undef SMDT_CAST
  return hipGetLastError();
}
