// Host-side AdamW for ZeRO optimizer offload (DeepSpeed cpu_adam equivalent, SURVEY P8/K10:
// `offload_optimizer.device: cpu` in
// /root/reference/4_training_alpaca_deepspeed/configs/default_offload_opt_param-original.json).
//
// The fp32 master shard and both moments live in pinned host memory; the reduced fp32 gradient
// shard arrives by D2H copy. One pass per element: moments, bias-corrected update, decoupled
// weight decay, and the bf16 (round-to-nearest-even) copy that is DMA'd back to HBM. Work is split
// into contiguous chunks over std::threads; the inner loop is written so GCC vectorises it
// (no aliasing, no branches).
#include <pybind11/pybind11.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>

namespace py = pybind11;

namespace {

inline uint16_t f32_to_bf16_rne(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  if ((u & 0x7f800000u) == 0x7f800000u && (u & 0x7fffffu)) return uint16_t((u >> 16) | 0x40);  // NaN
  u += 0x7fffu + ((u >> 16) & 1u);
  return uint16_t(u >> 16);
}

struct AdamArgs {
  float* __restrict__ p;
  const float* __restrict__ g;
  float* __restrict__ m;
  float* __restrict__ v;
  uint16_t* __restrict__ out_bf16;  // may be null
  float lr, b1, b2, eps, wd, bc1, bc2, gmul;
  bool adamw;
};

void adam_range(const AdamArgs& a, int64_t s, int64_t e) {
  const float step = a.lr / a.bc1;
  const float ib2 = 1.f / std::sqrt(a.bc2);
  const float dec = a.adamw ? (1.f - a.lr * a.wd) : 1.f;
  const float l2 = a.adamw ? 0.f : a.wd;
  float* __restrict__ p = a.p;
  const float* __restrict__ g = a.g;
  float* __restrict__ m = a.m;
  float* __restrict__ v = a.v;
  for (int64_t i = s; i < e; ++i) {
    float gi = g[i] * a.gmul + l2 * p[i];
    float mi = a.b1 * m[i] + (1.f - a.b1) * gi;
    float vi = a.b2 * v[i] + (1.f - a.b2) * gi * gi;
    m[i] = mi;
    v[i] = vi;
    p[i] = p[i] * dec - step * mi / (std::sqrt(vi) * ib2 + a.eps);
  }
  if (a.out_bf16)
    for (int64_t i = s; i < e; ++i) a.out_bf16[i] = f32_to_bf16_rne(p[i]);
}

void cpu_adam(uintptr_t p, uintptr_t g, uintptr_t m, uintptr_t v, uintptr_t out_bf16, int64_t n, float lr,
              float b1, float b2, float eps, float wd, int64_t step, bool adamw, float grad_mul, int threads) {
  AdamArgs a{reinterpret_cast<float*>(p), reinterpret_cast<const float*>(g), reinterpret_cast<float*>(m),
             reinterpret_cast<float*>(v), reinterpret_cast<uint16_t*>(out_bf16), lr, b1, b2, eps, wd,
             float(1.0 - std::pow(double(b1), double(step))), float(1.0 - std::pow(double(b2), double(step))),
             grad_mul, adamw};
  py::gil_scoped_release nogil;
  int T = threads > 0 ? threads : int(std::max(1u, std::thread::hardware_concurrency()));
  T = int(std::min<int64_t>(T, std::max<int64_t>(1, n / (1 << 16))));
  if (T <= 1) {
    adam_range(a, 0, n);
    return;
  }
  std::vector<std::thread> th;
  const int64_t chunk = ((n + T - 1) / T + 15) / 16 * 16;
  for (int t = 0; t < T; ++t) {
    int64_t s = t * chunk, e = std::min(n, s + chunk);
    if (s >= e) break;
    th.emplace_back(adam_range, std::cref(a), s, e);
  }
  for (auto& x : th) x.join();
}

double cpu_sumsq(uintptr_t g, int64_t n) {
  const float* x = reinterpret_cast<const float*>(g);
  py::gil_scoped_release nogil;
  double acc = 0.0;
  for (int64_t i = 0; i < n; ++i) acc += double(x[i]) * double(x[i]);
  return acc;
}

}  // namespace

void register_cpu_adam(py::module_& m) {
  m.def("cpu_adam", &cpu_adam, py::arg("param"), py::arg("grad"), py::arg("exp_avg"), py::arg("exp_avg_sq"),
        py::arg("out_bf16"), py::arg("n"), py::arg("lr"), py::arg("beta1"), py::arg("beta2"), py::arg("eps"),
        py::arg("weight_decay"), py::arg("step"), py::arg("adamw"), py::arg("grad_mul"), py::arg("threads") = 0,
        "In-place AdamW on host fp32 buffers (raw pointers); optional bf16 RNE copy of the params.");
  m.def("cpu_sumsq", &cpu_sumsq, py::arg("grad"), py::arg("n"));
}
