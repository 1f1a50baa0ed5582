// PyTorch bindings for the gfx950 kernel library (module `smdt_amd._C`).
//
// This is the only translation unit that sees ATen. Each binding validates shapes / dtypes /
// contiguity on the host (a kernel is never launched on operands it does not expect), allocates
// outputs through the caching allocator, and forwards raw pointers plus the current HIP stream
// to the C launchers in kernels/launchers.h.
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>
#include <c10/hip/HIPGuard.h>

#include "kernels/launchers.h"

namespace {

using torch::Tensor;
using OptT = std::optional<Tensor>;

hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

int dcode(const Tensor& t) {
  switch (t.scalar_type()) {
    case at::kFloat: return 0;
    case at::kBFloat16: return 1;
    case at::kHalf: return 2;
    default: TORCH_CHECK(false, "smdt_amd: unsupported dtype ", t.scalar_type());
  }
}

void check(hipError_t e, const char* what) {
  TORCH_CHECK(e == hipSuccess, "smdt_amd kernel '", what, "' failed: ", hipGetErrorString(e));
}

void need_cuda(const Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), "smdt_amd: '", name, "' must be a GPU tensor");
}

void need_contig(const Tensor& t, const char* name) {
  need_cuda(t, name);
  TORCH_CHECK(t.is_contiguous(), "smdt_amd: '", name, "' must be contiguous");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0, "smdt_amd: '", name,
              "' must be 16-byte aligned");
}

const void* optr(const OptT& t) { return t.has_value() ? t->data_ptr() : nullptr; }

// ------------------------------------------------------------------ LayerNorm / RMSNorm
// out_y (optional): a contiguous tensor of x's size and dtype the normalised output is written
// into — a slice of a sequence-parallel all-gather buffer, so the gather needs no local copy.
static Tensor out_or_new(const OptT& out, const Tensor& like, const char* n) {
  if (!out) return torch::empty_like(like);
  TORCH_CHECK(out->is_contiguous() && out->numel() == like.numel() && out->dtype() == like.dtype() &&
                  out->device() == like.device(),
              n, ": output buffer must be contiguous with the input's size, dtype and device");
  return out->view(like.sizes());
}

std::vector<Tensor> layernorm_fwd(Tensor x, OptT res, OptT bias, Tensor gamma, OptT beta,
                                  double eps, double p_drop, int64_t seed, int64_t offset,
                                  bool rms, bool want_s, OptT out_y, OptT x2) {
  need_contig(x, "x");
  need_contig(gamma, "gamma");
  const int64_t H = x.size(-1);
  const int64_t rows = x.numel() / H;
  TORCH_CHECK(gamma.numel() == H, "layernorm: gamma size mismatch");
  if (res) { need_contig(*res, "residual"); TORCH_CHECK(res->sizes() == x.sizes() && res->dtype() == x.dtype(), "layernorm: residual mismatch"); }
  if (bias) { need_contig(*bias, "bias"); TORCH_CHECK(bias->numel() == H && bias->dtype() == gamma.dtype(), "layernorm: bias mismatch"); }
  if (beta) { need_contig(*beta, "beta"); TORCH_CHECK(beta->numel() == H && beta->dtype() == gamma.dtype(), "layernorm: beta mismatch"); }
  if (x2) { need_contig(*x2, "x2"); TORCH_CHECK(x2->sizes() == x.sizes() && x2->dtype() == x.dtype(), "layernorm: x2 mismatch"); }
  auto y = out_or_new(out_y, x, "layernorm_fwd");
  Tensor s;
  const bool make_s = want_s || res.has_value() || bias.has_value() || p_drop > 0.0 || x2.has_value();
  if (make_s) s = torch::empty_like(x);
  auto f32 = x.options().dtype(at::kFloat);
  auto mean = torch::empty({rows}, f32);
  auto rstd = torch::empty({rows}, f32);
  check(smdt_layernorm_fwd(dcode(x), dcode(gamma), x.data_ptr(), optr(res), optr(bias),
                           gamma.data_ptr(), optr(beta), y.data_ptr(),
                           make_s ? s.data_ptr() : nullptr, mean.data_ptr<float>(),
                           rstd.data_ptr<float>(), rows, (int)H, (float)eps, (float)p_drop,
                           (uint64_t)seed, (uint64_t)offset, rms ? 1 : 0, optr(x2), cur_stream()),
        "layernorm_fwd");
  return {y, make_s ? s : x, mean, rstd};
}

// dgamma_acc / dbeta_acc / dbias_acc (optional): fp32 [H] buffers (DDP main_grad views) the
// parameter gradients are ACCUMULATED into instead of being returned.
static Tensor acc_target(const OptT& t, int64_t H, const char* n) {
  if (!t) return Tensor();
  TORCH_CHECK(t->scalar_type() == at::kFloat && t->is_contiguous() && t->numel() == H, n,
              ": accumulate target must be a contiguous fp32 tensor of ", H, " elements");
  return *t;
}

std::vector<Tensor> layernorm_bwd(Tensor dy, OptT ds_in, Tensor s, Tensor gamma, Tensor mean,
                                  Tensor rstd, double p_drop, int64_t seed, int64_t offset,
                                  bool rms, bool want_dx, bool want_dbias, OptT dgamma_acc,
                                  OptT dbeta_acc, OptT dbias_acc, OptT out_dx, OptT dy2) {
  need_contig(dy, "dy");
  need_contig(s, "s");
  need_contig(gamma, "gamma");
  const int64_t H = s.size(-1);
  const int64_t rows = s.numel() / H;
  TORCH_CHECK(dy.sizes() == s.sizes() && dy.dtype() == s.dtype(), "layernorm_bwd: dy mismatch");
  if (ds_in) { need_contig(*ds_in, "ds_in"); TORCH_CHECK(ds_in->sizes() == s.sizes() && ds_in->dtype() == s.dtype(), "layernorm_bwd: ds_in mismatch"); }
  if (dy2) { need_contig(*dy2, "dy2"); TORCH_CHECK(dy2->sizes() == s.sizes() && dy2->dtype() == s.dtype(), "layernorm_bwd: dy2 mismatch"); }
  // out_dx (optional): where dx goes (a slice of an all-gather buffer, see layernorm_fwd); without
  // dropout dx IS ds, so ds lands there too
  const bool sep = want_dx && p_drop > 0.0;
  auto ds = (out_dx && !sep) ? out_or_new(out_dx, s, "layernorm_bwd") : torch::empty_like(s);
  Tensor dx = sep ? out_or_new(out_dx, s, "layernorm_bwd") : ds;
  const int nb = smdt_ln_bwd_nblocks(rows, (int)H);
  auto f32 = s.options().dtype(at::kFloat);
  auto partials = torch::empty({nb, 3, H}, f32);
  Tensor ga = acc_target(dgamma_acc, H, "dgamma_acc"), ba = acc_target(dbeta_acc, H, "dbeta_acc"),
         bia = acc_target(dbias_acc, H, "dbias_acc");
  const int acc_mask = (ga.defined() ? 1 : 0) | (ba.defined() ? 2 : 0) | (bia.defined() ? 4 : 0);
  auto dgamma = ga.defined() ? ga : torch::empty({H}, f32);
  Tensor dbeta = rms ? Tensor() : (ba.defined() ? ba : torch::empty({H}, f32));
  Tensor dbias = want_dbias ? (bia.defined() ? bia : torch::empty({H}, f32)) : Tensor();
  check(smdt_layernorm_bwd(dcode(s), dcode(gamma), dy.data_ptr(), optr(ds_in), s.data_ptr(),
                           gamma.data_ptr(), rms ? nullptr : mean.data_ptr<float>(),
                           rstd.data_ptr<float>(), ds.data_ptr(), dx.data_ptr(),
                           partials.data_ptr<float>(), nb, dgamma.data_ptr<float>(),
                           rms ? nullptr : dbeta.data_ptr<float>(),
                           want_dbias ? dbias.data_ptr<float>() : nullptr, rows, (int)H,
                           (float)p_drop, (uint64_t)seed, (uint64_t)offset, rms ? 1 : 0, acc_mask,
                           optr(dy2), cur_stream()),
        "layernorm_bwd");
  return {ds, dx, dgamma, rms ? dgamma.new_empty({0}) : dbeta,
          want_dbias ? dbias : dgamma.new_empty({0})};
}

// ------------------------------------------------------------------ bias + activation
Tensor bias_act_fwd(Tensor x, OptT bias, int64_t act) {
  need_contig(x, "x");
  const int64_t N = x.size(-1), rows = x.numel() / N;
  if (bias) { need_contig(*bias, "bias"); TORCH_CHECK(bias->numel() == N && bias->dtype() == x.dtype(), "bias_act: bias mismatch"); }
  auto y = torch::empty_like(x);
  check(smdt_bias_act_fwd(dcode(x), (int)act, x.data_ptr(), optr(bias), y.data_ptr(), rows, (int)N,
                          cur_stream()),
        "bias_act_fwd");
  return y;
}

std::vector<Tensor> bias_act_bwd(Tensor dy, Tensor x, OptT bias, int64_t act, bool want_dbias,
                                 OptT dbias_acc) {
  need_contig(dy, "dy");
  need_contig(x, "x");
  TORCH_CHECK(dy.sizes() == x.sizes() && dy.dtype() == x.dtype(), "bias_act_bwd: shape mismatch");
  const int64_t N = x.size(-1), rows = x.numel() / N;
  auto dx = torch::empty_like(x);
  Tensor part, dbias;
  if (want_dbias) {
    const int slices = smdt_bias_act_slices(rows, (int)N);
    part = torch::empty({slices, N}, x.options().dtype(at::kFloat));
    dbias = dbias_acc ? acc_target(dbias_acc, N, "dbias_acc") : torch::empty({N}, x.options().dtype(at::kFloat));
  }
  check(smdt_bias_act_bwd(dcode(x), (int)act, dy.data_ptr(), x.data_ptr(), optr(bias),
                          dx.data_ptr(), want_dbias ? part.data_ptr<float>() : nullptr,
                          want_dbias ? dbias.data_ptr<float>() : nullptr, rows, (int)N,
                          dbias_acc ? 1 : 0, cur_stream()),
        "bias_act_bwd");
  return {dx, want_dbias ? dbias : dx.new_empty({0})};
}

Tensor swiglu_fwd(Tensor x) {
  need_contig(x, "x");
  const int64_t F2 = x.size(-1), rows = x.numel() / F2;
  TORCH_CHECK(F2 % 2 == 0, "swiglu: last dim must be even");
  auto sizes = x.sizes().vec();
  sizes.back() = F2 / 2;
  auto y = torch::empty(sizes, x.options());
  check(smdt_swiglu_fwd(dcode(x), x.data_ptr(), y.data_ptr(), rows, (int)(F2 / 2), cur_stream()),
        "swiglu_fwd");
  return y;
}

Tensor swiglu_bwd(Tensor dy, Tensor x) {
  need_contig(dy, "dy");
  need_contig(x, "x");
  const int64_t F2 = x.size(-1), rows = x.numel() / F2;
  TORCH_CHECK(dy.numel() * 2 == x.numel(), "swiglu_bwd: shape mismatch");
  auto dx = torch::empty_like(x);
  check(smdt_swiglu_bwd(dcode(x), dy.data_ptr(), x.data_ptr(), dx.data_ptr(), rows, (int)(F2 / 2),
                        cur_stream()),
        "swiglu_bwd");
  return dx;
}

// ------------------------------------------------------------------ masked softmax
Tensor softmax_fwd(Tensor x, OptT mask, int64_t mode, double scale) {
  need_contig(x, "x");
  TORCH_CHECK(x.dim() == 4, "softmax: expects [b, np, sq, sk]");
  const int64_t sk = x.size(3), sq = x.size(2), heads = x.size(1);
  const int64_t rows = x.numel() / sk;
  if (mode == 2) {
    TORCH_CHECK(mask.has_value(), "softmax: mode 2 needs a mask");
    need_contig(*mask, "mask");
    TORCH_CHECK(mask->scalar_type() == at::kBool || mask->scalar_type() == at::kByte, "softmax: mask must be bool/uint8");
    TORCH_CHECK(mask->numel() == x.size(0) * sq * sk, "softmax: mask must be [b, 1, sq, sk]");
  }
  auto y = torch::empty_like(x);
  check(smdt_softmax_fwd(dcode(x), (int)mode, x.data_ptr(),
                         mode == 2 ? (const uint8_t*)mask->data_ptr() : nullptr, y.data_ptr(), rows,
                         (int)sq, (int)sk, (int)heads, (float)scale, cur_stream()),
        "softmax_fwd");
  return y;
}

Tensor softmax_bwd(Tensor dy, Tensor y, int64_t mode, double scale) {
  need_contig(dy, "dy");
  need_contig(y, "y");
  TORCH_CHECK(dy.sizes() == y.sizes(), "softmax_bwd: shape mismatch");
  const int64_t sk = y.size(3), sq = y.size(2), rows = y.numel() / sk;
  auto dx = torch::empty_like(y);
  check(smdt_softmax_bwd(dcode(y), (int)mode, dy.data_ptr(), y.data_ptr(), dx.data_ptr(), rows,
                         (int)sq, (int)sk, (float)scale, cur_stream()),
        "softmax_bwd");
  return dx;
}

// ------------------------------------------------------------------ graph-safe dropout RNG
// counter: a persistent device int32 [1] (None: off). While set, every dropout kernel (flash
// attention, fused LayerNorm) mixes *counter into its keys at run time; the training step
// advances it on the device, so HIP-graph replays of a captured step draw fresh masks.
static Tensor g_rng_counter;
void set_rng_step(OptT counter) {
  if (counter) {
    TORCH_CHECK(counter->is_cuda() && counter->scalar_type() == at::kInt && counter->numel() == 1,
                "set_rng_step: device int32 [1] counter");
    g_rng_counter = *counter;
    smdt_set_rng_step(reinterpret_cast<uint32_t*>(counter->data_ptr<int>()));
  } else {
    g_rng_counter = Tensor();
    smdt_set_rng_step(nullptr);
  }
}

// ------------------------------------------------------------------ optimizer
void adam(Tensor master, Tensor grad, Tensor m, Tensor v, OptT model_out, double lr, double beta1,
          double beta2, double eps, double wd, int64_t step, bool adamw, OptT grad_mul,
          OptT found_inf) {
  for (auto* t : {&master, &grad, &m, &v}) {
    need_contig(*t, "adam buffer");
    TORCH_CHECK(t->scalar_type() == at::kFloat, "adam: fp32 buffers expected");
    TORCH_CHECK(t->numel() == master.numel(), "adam: buffer size mismatch");
  }
  int mdt = 0;
  if (model_out) {
    need_contig(*model_out, "model_out");
    TORCH_CHECK(model_out->numel() == master.numel(), "adam: model_out size mismatch");
    mdt = dcode(*model_out);
    TORCH_CHECK(mdt != 0, "adam: model_out must be bf16/fp16 (fp32 masters ARE the model)");
  }
  if (grad_mul) TORCH_CHECK(grad_mul->scalar_type() == at::kFloat && grad_mul->is_cuda(), "adam: grad_mul fp32 scalar");
  if (found_inf) TORCH_CHECK(found_inf->scalar_type() == at::kInt && found_inf->is_cuda(), "adam: found_inf int32 scalar");
  const double bc1 = 1.0 - std::pow(beta1, (double)step);
  const double bc2 = 1.0 - std::pow(beta2, (double)step);
  check(smdt_adam(master.data_ptr<float>(), grad.data_ptr<float>(), m.data_ptr<float>(),
                  v.data_ptr<float>(), model_out ? model_out->data_ptr() : nullptr, mdt,
                  master.numel(), (float)lr, (float)beta1, (float)beta2, (float)eps, (float)wd,
                  (float)bc1, (float)bc2, adamw ? 1 : 0,
                  grad_mul ? grad_mul->data_ptr<float>() : nullptr,
                  found_inf ? found_inf->data_ptr<int>() : nullptr, nullptr, cur_stream()),
        "adam");
}

// HIP-graph capturable form: lr and the bias corrections come from the device tensor
// hyper = [lr, 1 - beta1^t, 1 - beta2^t] (fp32, updated on the device each step), so a captured
// step replays with the current step count and learning rate.
void adam_capturable(Tensor master, Tensor grad, Tensor m, Tensor v, OptT model_out, Tensor hyper,
                     double beta1, double beta2, double eps, double wd, bool adamw, OptT grad_mul,
                     OptT found_inf) {
  for (auto* t : {&master, &grad, &m, &v}) {
    need_contig(*t, "adam buffer");
    TORCH_CHECK(t->scalar_type() == at::kFloat, "adam: fp32 buffers expected");
    TORCH_CHECK(t->numel() == master.numel(), "adam: buffer size mismatch");
  }
  TORCH_CHECK(hyper.scalar_type() == at::kFloat && hyper.is_cuda() && hyper.numel() == 3 && hyper.is_contiguous(),
              "adam_capturable: hyper = device fp32 [lr, bc1, bc2]");
  int mdt = 0;
  if (model_out) {
    need_contig(*model_out, "model_out");
    TORCH_CHECK(model_out->numel() == master.numel(), "adam: model_out size mismatch");
    mdt = dcode(*model_out);
    TORCH_CHECK(mdt != 0, "adam: model_out must be bf16/fp16 (fp32 masters ARE the model)");
  }
  if (grad_mul) TORCH_CHECK(grad_mul->scalar_type() == at::kFloat && grad_mul->is_cuda(), "adam: grad_mul fp32 scalar");
  if (found_inf) TORCH_CHECK(found_inf->scalar_type() == at::kInt && found_inf->is_cuda(), "adam: found_inf int32 scalar");
  check(smdt_adam(master.data_ptr<float>(), grad.data_ptr<float>(), m.data_ptr<float>(),
                  v.data_ptr<float>(), model_out ? model_out->data_ptr() : nullptr, mdt,
                  master.numel(), 0.f, (float)beta1, (float)beta2, (float)eps, (float)wd, 1.f, 1.f,
                  adamw ? 1 : 0, grad_mul ? grad_mul->data_ptr<float>() : nullptr,
                  found_inf ? found_inf->data_ptr<int>() : nullptr, hyper.data_ptr<float>(), cur_stream()),
        "adam_capturable");
}

Tensor sumsq(Tensor x, OptT found_inf) {
  need_contig(x, "x");
  const int64_t n = x.numel();
  const int nb = smdt_sumsq_nblocks(n);
  auto f32 = x.options().dtype(at::kFloat);
  auto partial = torch::empty({nb}, f32);
  auto out = torch::empty({1}, f32);
  if (found_inf) TORCH_CHECK(found_inf->scalar_type() == at::kInt && found_inf->is_cuda(), "sumsq: found_inf int32");
  check(smdt_sumsq(dcode(x), x.data_ptr(), n, partial.data_ptr<float>(), nb, out.data_ptr<float>(),
                   found_inf ? found_inf->data_ptr<int>() : nullptr, cur_stream()),
        "sumsq");
  return out;
}

std::vector<Tensor> clip_coef(Tensor sumsq_t, double max_norm, double inv_scale) {
  TORCH_CHECK(sumsq_t.scalar_type() == at::kFloat && sumsq_t.is_cuda(), "clip_coef: fp32 scalar");
  auto mul = torch::empty({1}, sumsq_t.options());
  auto norm = torch::empty({1}, sumsq_t.options());
  check(smdt_clip_coef(sumsq_t.data_ptr<float>(), (float)max_norm, (float)inv_scale,
                       mul.data_ptr<float>(), norm.data_ptr<float>(), cur_stream()),
        "clip_coef");
  return {mul, norm};
}

void scale_(Tensor x, OptT mul, double cmul) {
  need_contig(x, "x");
  check(smdt_scale(dcode(x), x.data_ptr(), x.numel(), mul ? mul->data_ptr<float>() : nullptr,
                   (float)cmul, cur_stream()),
        "scale");
}

void cast_(Tensor x, Tensor y, bool accumulate) {
  need_contig(x, "x");
  need_contig(y, "y");
  TORCH_CHECK(x.numel() == y.numel(), "cast: size mismatch");
  check(smdt_cast(dcode(x), dcode(y), x.data_ptr(), y.data_ptr(), x.numel(), accumulate ? 1 : 0,
                  cur_stream()),
        "cast");
}

// ------------------------------------------------------------------ augmentation filters (fp32)
// y [N, C, H, W] = x (*) k[n] per sample (reflect padding); k [N, KS, KS], KS in {3, 5, 7}.
Tensor aug_depthwise(Tensor x, Tensor k) {
  TORCH_CHECK(x.is_cuda() && k.is_cuda() && x.scalar_type() == at::kFloat && k.scalar_type() == at::kFloat,
              "aug_depthwise: fp32 GPU tensors");
  TORCH_CHECK(x.dim() == 4 && k.dim() == 3 && k.size(0) == x.size(0) && k.size(1) == k.size(2), "aug_depthwise: shapes");
  x = x.contiguous();
  k = k.contiguous();
  auto y = torch::empty_like(x);
  check(smdt_aug_depthwise(x.data_ptr<float>(), k.data_ptr<float>(), y.data_ptr<float>(), (int)x.size(0),
                           (int)x.size(1), (int)x.size(2), (int)x.size(3), (int)k.size(1), cur_stream()),
        "aug_depthwise");
  return y;
}

// y = 3 x 3 median of every channel of x [N, C, H, W] (reflect padding).
Tensor aug_median3(Tensor x) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kFloat && x.dim() == 4, "aug_median3: fp32 [N, C, H, W] GPU tensor");
  x = x.contiguous();
  auto y = torch::empty_like(x);
  check(smdt_aug_median3(x.data_ptr<float>(), y.data_ptr<float>(), (int)(x.size(0) * x.size(1)), (int)x.size(2),
                         (int)x.size(3), cur_stream()),
        "aug_median3");
  return y;
}

// ------------------------------------------------------------------ row gather with zero fill
// out[r] = map[r] >= 0 ? src[map[r]] : 0; src [Ns, ...] contiguous, map int64 [Nd] on the device
Tensor gather_rows(Tensor src, Tensor map) {
  need_contig(src, "src");
  need_contig(map, "map");
  TORCH_CHECK(map.scalar_type() == at::kLong && map.dim() == 1 && map.device() == src.device(),
              "gather_rows: map must be a 1-D int64 tensor on src's device");
  TORCH_CHECK(src.dim() >= 1, "gather_rows: src must have a row dimension");
  const int64_t rb = src.numel() / std::max<int64_t>(src.size(0), 1) * src.element_size();
  TORCH_CHECK(rb % 16 == 0, "gather_rows: row bytes must be a multiple of 16");
  auto sizes = src.sizes().vec();
  sizes[0] = map.size(0);
  auto out = torch::empty(sizes, src.options());
  check(smdt_gather_rows(src.data_ptr(), map.data_ptr<int64_t>(), out.data_ptr(), map.size(0), src.size(0), rb,
                         cur_stream()),
        "gather_rows");
  return out;
}

// ------------------------------------------------------------------ 2-D transpose (16-bit)
// out [C, R] = x [R, C]^T, contiguous (feeds the dgrad GEMMs in the TN layout).
Tensor transpose2d(Tensor x) {
  need_contig(x, "x");
  TORCH_CHECK(x.dim() == 2, "transpose2d: x must be 2-D");
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 || x.scalar_type() == at::kHalf, "transpose2d: bf16 / fp16 only");
  TORCH_CHECK(x.size(0) % 8 == 0 && x.size(1) % 8 == 0, "transpose2d: both dims must be multiples of 8");
  auto out = torch::empty({x.size(1), x.size(0)}, x.options());
  check(smdt_transpose16(x.data_ptr(), out.data_ptr(), x.size(0), x.size(1), cur_stream()), "transpose2d");
  return out;
}

// ------------------------------------------------------------------ paced link stand-in
// recv <- send on `blocks` workgroups, held until `ns` have passed (comm/loopback.py)
void paced_copy(Tensor recv, Tensor send, int64_t blocks, int64_t ns) {
  need_contig(recv, "recv");
  need_contig(send, "send");
  TORCH_CHECK(recv.is_cuda() && send.is_cuda(), "paced_copy: CUDA tensors");
  const int64_t nb = send.numel() * send.element_size();
  TORCH_CHECK(nb == recv.numel() * recv.element_size() && nb % 16 == 0, "paced_copy: equal sizes, multiple of 16 B");
  TORCH_CHECK((uintptr_t)send.data_ptr() % 16 == 0 && (uintptr_t)recv.data_ptr() % 16 == 0, "paced_copy: 16-B aligned");
  check(smdt_paced_copy(send.data_ptr(), recv.data_ptr(), nb, (int)blocks, ns, cur_stream()), "paced_copy");
}

// ------------------------------------------------------------------ RoPE
// x: [ntok, nh, d] strided view (last dim contiguous), rotary applied in place to the first
// `rot` elements of each head.
void rope_(Tensor x, Tensor cos_t, Tensor sin_t, int64_t rot, int64_t pos_div, int64_t pos_mod,
           bool backward) {
  need_cuda(x, "x");
  TORCH_CHECK(x.dim() == 3 && x.stride(2) == 1, "rope: x must be [ntok, nh, d] with unit last stride");
  need_contig(cos_t, "cos");
  need_contig(sin_t, "sin");
  TORCH_CHECK(cos_t.scalar_type() == at::kFloat && sin_t.scalar_type() == at::kFloat, "rope: fp32 tables");
  TORCH_CHECK(rot <= x.size(2) && rot % 16 == 0 && cos_t.size(-1) == rot / 2, "rope: rotary dim mismatch");
  TORCH_CHECK(x.stride(0) % 8 == 0 && x.stride(1) % 8 == 0, "rope: strides must keep 16-byte alignment");
  check(smdt_rope(dcode(x), x.data_ptr(), x.size(0), (int)x.size(1), x.stride(0), x.stride(1),
                  (int)rot, cos_t.data_ptr<float>(), sin_t.data_ptr<float>(), (int)pos_div,
                  (int)pos_mod, backward ? 1 : 0, cur_stream()),
        "rope");
}

// ------------------------------------------------------------------ forward / dgrad GEMM (MFMA)
// out[M, N] = a[M, K] . b[N, K]^T with the epilogue `epi` (0 none, 1 + bias, 2 bias + GeLU-tanh:
// out = pre-activation, out2 = activation). Returns false (and does nothing) for an unsupported
// shape / layout so the caller can take the library GEMM; out / out2 may be given (e.g. a slice of
// a larger buffer), else they are allocated.
bool gemm_tn_supported(Tensor a, Tensor b) {
  if (!a.is_cuda() || !b.is_cuda() || a.dim() != 2 || b.dim() != 2 || !a.is_contiguous() || !b.is_contiguous()) return false;
  if ((a.scalar_type() != at::kBFloat16 && a.scalar_type() != at::kHalf) || b.scalar_type() != a.scalar_type()) return false;
  if (a.size(1) != b.size(1)) return false;
  if (reinterpret_cast<uintptr_t>(a.data_ptr()) % 16 || reinterpret_cast<uintptr_t>(b.data_ptr()) % 16) return false;
  return smdt_gemm_tn_supported(a.size(0), b.size(0), a.size(1)) != 0;
}

std::vector<Tensor> gemm_tn(Tensor a, Tensor b, int64_t epi, OptT bias, OptT out, OptT out2, int64_t max_blocks,
                            int64_t var, OptT aux) {
  TORCH_CHECK(gemm_tn_supported(a, b), "gemm_tn: unsupported operands");
  TORCH_CHECK(epi >= 0 && epi <= 3, "gemm_tn: epilogue");
  const int64_t M = a.size(0), N = b.size(0), K = a.size(1);
  if (epi >= 1) {
    TORCH_CHECK(bias.has_value(), "gemm_tn: the epilogue needs a bias");
    need_contig(*bias, "bias");
    TORCH_CHECK(bias->numel() == N && bias->scalar_type() == a.scalar_type(), "gemm_tn: bias mismatch");
  }
  if (epi == 3) {
    TORCH_CHECK(aux.has_value(), "gemm_tn: the GeLU-backward epilogue needs the pre-activation");
    need_contig(*aux, "aux");
    TORCH_CHECK(aux->numel() == M * N && aux->scalar_type() == a.scalar_type() && aux->device() == a.device(),
                "gemm_tn: pre-activation mismatch");
  }
  auto mk = [&](const OptT& o, const char* n) {
    if (!o) return torch::empty({M, N}, a.options());
    need_contig(*o, n);
    TORCH_CHECK(o->numel() == M * N && o->scalar_type() == a.scalar_type() && o->device() == a.device(),
                "gemm_tn: output buffer mismatch");
    return *o;
  };
  Tensor c = mk(out, "out");
  Tensor c2 = epi == 2 ? mk(out2, "out2") : Tensor();
  check(smdt_gemm_tn_var(dcode(a), (int)epi, a.data_ptr(), b.data_ptr(), c.data_ptr(),
                         epi == 2 ? c2.data_ptr() : nullptr, optr(bias), epi == 3 ? aux->data_ptr() : nullptr, M,
                         N, K, (int)max_blocks, (int)var, cur_stream()),
        "gemm_tn");
  if (epi == 2) return {c, c2};
  return {c};
}

// ------------------------------------------------------------------ weight gradient (MFMA)
// main_grad[N, K] (fp32) += dy[M, N]^T . x[M, K]; returns false when the shape is unsupported.
bool wgrad_mfma(Tensor main_grad, Tensor dy, Tensor x, int64_t max_splits) {
  if (!main_grad.is_cuda() || main_grad.scalar_type() != at::kFloat || !main_grad.is_contiguous()) return false;
  if (dy.dim() != 2 || x.dim() != 2 || !dy.is_contiguous() || !x.is_contiguous()) return false;
  if ((dy.scalar_type() != at::kBFloat16 && dy.scalar_type() != at::kHalf) || x.scalar_type() != dy.scalar_type())
    return false;
  const int64_t M = dy.size(0), N = dy.size(1), K = x.size(1);
  if (x.size(0) != M || main_grad.numel() != N * K || !smdt_wgrad_supported(M, N, K)) return false;
  check(smdt_wgrad_accumulate_t(dcode(dy), dy.data_ptr(), x.data_ptr(), main_grad.data_ptr<float>(), M, N, K, (int)max_splits,
                              cur_stream()),
        "wgrad_mfma");
  return true;
}

// Grouped form: main_grads[i] += dys[i]^T . xs[i] for every i in ONE launch per 32 problems.
// Returns false (and does nothing) when any problem is unsupported. The targets must not overlap.
// ``biases`` (optional, one per problem; an empty tensor = none): fp32 [N] targets that receive
// the column sums of dy — the bias gradient — from the same launch.
// overwrite (optional, per problem): the main_grad holds no data yet (a lazily zeroed gradient
// buffer): the kernel stores dy^T x instead of adding it (no read of the target).
bool wgrad_grouped(std::vector<Tensor> main_grads, std::vector<Tensor> dys, std::vector<Tensor> xs,
                   std::vector<Tensor> biases, std::vector<bool> overwrite, int64_t cus) {
  const size_t n = main_grads.size();
  TORCH_CHECK(dys.size() == n && xs.size() == n, "wgrad_grouped: list lengths differ");
  TORCH_CHECK(biases.empty() || biases.size() == n, "wgrad_grouped: biases list length");
  TORCH_CHECK(overwrite.empty() || overwrite.size() == n, "wgrad_grouped: overwrite list length");
  std::vector<SmdtWgradProblem> probs(n);
  for (size_t i = 0; i < n; ++i) {
    const Tensor &mg = main_grads[i], &dy = dys[i], &x = xs[i];
    if (!mg.is_cuda() || mg.scalar_type() != at::kFloat || !mg.is_contiguous()) return false;
    if (dy.dim() != 2 || x.dim() != 2 || !dy.is_contiguous() || !x.is_contiguous()) return false;
    if ((dy.scalar_type() != at::kBFloat16 && dy.scalar_type() != at::kHalf) || x.scalar_type() != dy.scalar_type() ||
        dy.scalar_type() != dys[0].scalar_type())
      return false;
    if (dy.get_device() != mg.get_device() || x.get_device() != mg.get_device()) return false;
    const int64_t M = dy.size(0), N = dy.size(1), K = x.size(1);
    if (x.size(0) != M || mg.numel() != N * K || !smdt_wgrad_supported(M, N, K)) return false;
    float* bg = nullptr;
    if (!biases.empty() && biases[i].numel() > 0) {
      const Tensor& bt = biases[i];
      if (!bt.is_cuda() || bt.scalar_type() != at::kFloat || !bt.is_contiguous() || bt.numel() != N ||
          bt.get_device() != mg.get_device())
        return false;
      bg = bt.data_ptr<float>();
    }
    probs[i] = SmdtWgradProblem{dy.data_ptr(), x.data_ptr(), mg.data_ptr<float>(), M, N, K, bg,
                                (!overwrite.empty() && overwrite[i]) ? 1 : 0};
  }
  if (n == 0) return true;
  check(smdt_wgrad_grouped_cus(dcode(dys[0]), probs.data(), (int)n, (int)cus, cur_stream()), "wgrad_grouped");
  return true;
}

// ------------------------------------------------------------------ bias gradient
// out[N] (fp32) = / += column sums of dy [.., N]
void bias_grad(Tensor dy, Tensor out, bool accumulate) {
  need_contig(dy, "dy");
  const int64_t N = dy.size(-1), rows = dy.numel() / N;
  Tensor o = acc_target(out, N, "bias_grad out");
  const int slices = smdt_bias_act_slices(rows, (int)N);
  auto part = torch::empty({slices, N}, dy.options().dtype(at::kFloat));
  check(smdt_bias_grad(dcode(dy), dy.data_ptr(), rows, (int)N, part.data_ptr<float>(),
                       o.data_ptr<float>(), accumulate ? 1 : 0, cur_stream()),
        "bias_grad");
}

// ------------------------------------------------------------------ cross entropy
// loss[rows] fp32; logits (16-bit, [rows, V]) are overwritten with softmax - onehot
Tensor ce_fused(Tensor logits, Tensor target, int64_t ignore_index, int64_t vvalid) {
  need_contig(logits, "logits");
  need_contig(target, "target");
  TORCH_CHECK(target.scalar_type() == at::kLong, "ce_fused: int64 targets");
  const int64_t V = logits.size(-1), rows = logits.numel() / V;
  TORCH_CHECK(target.numel() == rows, "ce_fused: target size mismatch");
  auto loss = torch::empty({rows}, logits.options().dtype(at::kFloat));
  check(smdt_ce_fused(dcode(logits), logits.data_ptr(), target.data_ptr<int64_t>(), loss.data_ptr<float>(),
                      rows, (int)V, (int)(vvalid > 0 ? vvalid : V), ignore_index, 0, 0, cur_stream()),
        "ce_fused");
  return loss;
}

// Vocab-parallel form: logits [rows, V] = this rank's vocab slice starting at vstart, overwritten
// with exp(x - m_local); returns stats [3, rows] fp32 = (m_local, sum, target logit or 0).
Tensor ce_fused_local(Tensor logits, Tensor target, int64_t vstart, int64_t vvalid) {
  need_contig(logits, "logits");
  need_contig(target, "target");
  TORCH_CHECK(target.scalar_type() == at::kLong, "ce_fused_local: int64 targets");
  const int64_t V = logits.size(-1), rows = logits.numel() / V;
  TORCH_CHECK(target.numel() == rows, "ce_fused_local: target size mismatch");
  auto stats = torch::empty({3, rows}, logits.options().dtype(at::kFloat));
  check(smdt_ce_fused(dcode(logits), logits.data_ptr(), target.data_ptr<int64_t>(), stats.data_ptr<float>(),
                      rows, (int)V, (int)(vvalid > 0 ? vvalid : V), -100, 1, vstart, cur_stream()),
        "ce_fused_local");
  return stats;
}

std::vector<Tensor> ce_stats(Tensor logits, Tensor target, int64_t vstart, int64_t vvalid) {
  need_contig(logits, "logits");
  need_contig(target, "target");
  TORCH_CHECK(target.scalar_type() == at::kLong, "ce: int64 targets");
  const int64_t V = logits.size(-1), rows = logits.numel() / V;
  TORCH_CHECK(target.numel() == rows, "ce: target size mismatch");
  auto f32 = logits.options().dtype(at::kFloat);
  auto mx = torch::empty({rows}, f32), se = torch::empty({rows}, f32), tg = torch::empty({rows}, f32);
  check(smdt_ce_stats(dcode(logits), logits.data_ptr(), target.data_ptr<int64_t>(), rows, (int)V,
                      (int)(vvalid > 0 ? vvalid : V), vstart, mx.data_ptr<float>(), se.data_ptr<float>(), tg.data_ptr<float>(),
                      cur_stream()),
        "ce_stats");
  return {mx, se, tg};
}

void ce_bwd(Tensor logits, Tensor target, Tensor gmax, Tensor gsum, Tensor dloss, Tensor out,
            int64_t vstart, int64_t ignore_index, int64_t vvalid) {
  need_contig(logits, "logits");
  need_contig(out, "dlogits");
  TORCH_CHECK(out.sizes() == logits.sizes() && out.dtype() == logits.dtype(), "ce_bwd: out mismatch");
  const int64_t V = logits.size(-1), rows = logits.numel() / V;
  for (auto* t : {&gmax, &gsum, &dloss}) {
    need_contig(*t, "ce row stat");
    TORCH_CHECK(t->scalar_type() == at::kFloat && t->numel() == rows, "ce_bwd: fp32 [rows] stats");
  }
  check(smdt_ce_bwd(dcode(logits), logits.data_ptr(), target.data_ptr<int64_t>(),
                    gmax.data_ptr<float>(), gsum.data_ptr<float>(), dloss.data_ptr<float>(),
                    out.data_ptr(), rows, (int)V, (int)(vvalid > 0 ? vvalid : V), vstart,
                    ignore_index, cur_stream()),
        "ce_bwd");
}

// ------------------------------------------------------------------ flash attention
// q: [B, S, H, D], k/v: [B, S, Hkv, D] (unit last stride, any other strides).
void fa_check(const Tensor& t, const char* n) {
  need_cuda(t, n);
  TORCH_CHECK(t.dim() == 4 && t.stride(3) == 1, "flash: '", n, "' must be [B, S, H, D] with unit last stride");
  TORCH_CHECK(t.scalar_type() == at::kBFloat16 || t.scalar_type() == at::kHalf, "flash: bf16 / fp16 only");
  TORCH_CHECK(t.stride(0) % 8 == 0 && t.stride(1) % 8 == 0 && t.stride(2) % 8 == 0 &&
                  reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0,
              "flash: '", n, "' must keep 16-byte row alignment");
}

// `out` (optional) is a preallocated [B, S, H, D] view with any strides (e.g. the [s, b, h]
// activation layout used by the transformer trunk).
std::vector<Tensor> flash_fwd(Tensor q, Tensor k, Tensor v, double scale, bool causal, OptT out,
                              double dropout_p, int64_t seed, int64_t offset) {
  fa_check(q, "q"); fa_check(k, "k"); fa_check(v, "v");
  TORCH_CHECK(k.scalar_type() == q.scalar_type() && v.scalar_type() == q.scalar_type(), "flash: q/k/v dtypes differ");
  const int64_t B = q.size(0), S = q.size(1), H = q.size(2), D = q.size(3), Hkv = k.size(2);
  TORCH_CHECK(k.size(0) == B && k.size(1) == S && k.size(3) == D && v.sizes() == k.sizes(), "flash: k/v shape mismatch");
  TORCH_CHECK((D == 64 || D == 128) && S % 128 == 0 && H % Hkv == 0, "flash: needs D in {64,128}, S % 128 == 0, H % Hkv == 0");
  Tensor o;
  if (out) {
    o = *out;
    fa_check(o, "out");
    TORCH_CHECK(o.sizes() == q.sizes(), "flash: out shape mismatch");
  } else {
    o = torch::empty({B, S, H, D}, q.options());
  }
  auto lse = torch::empty({B, H, S}, q.options().dtype(at::kFloat));
  TORCH_CHECK(o.scalar_type() == q.scalar_type(), "flash: out dtype mismatch");
  check(smdt_flash_fwd(dcode(q), q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), lse.data_ptr<float>(),
                       (int)B, (int)H, (int)Hkv, (int)S, (int)D, q.stride(0), q.stride(1), q.stride(2),
                       k.stride(0), k.stride(1), k.stride(2), v.stride(0), v.stride(1), v.stride(2),
                       o.stride(0), o.stride(1), o.stride(2), (float)scale, causal ? 1 : 0, (float)dropout_p,
                       (uint64_t)seed, (uint64_t)offset, cur_stream()),
        "flash_fwd");
  return {o, lse};
}

// dq / dk / dv (optional) are preallocated [B, S, H(kv), D] views with any strides, typically
// views into one fused d(QKV) buffer so the QKV projection backward needs no concatenation.
std::vector<Tensor> flash_bwd(Tensor q, Tensor k, Tensor v, Tensor o, Tensor dout, Tensor lse,
                              double scale, bool causal, OptT dq_out, OptT dk_out, OptT dv_out,
                              double dropout_p, int64_t seed, int64_t offset) {
  fa_check(q, "q"); fa_check(k, "k"); fa_check(v, "v"); fa_check(o, "o");
  TORCH_CHECK(k.scalar_type() == q.scalar_type() && v.scalar_type() == q.scalar_type() &&
              o.scalar_type() == q.scalar_type() && dout.scalar_type() == q.scalar_type(), "flash_bwd: dtypes differ");
  const int64_t B = q.size(0), S = q.size(1), H = q.size(2), D = q.size(3), Hkv = k.size(2);
  TORCH_CHECK((D == 64 || D == 128) && S % 128 == 0 && H % Hkv == 0, "flash_bwd: unsupported shape");
  TORCH_CHECK(dout.sizes() == o.sizes(), "flash_bwd: dout shape mismatch");
  if (dout.stride(3) != 1 || dout.stride(0) % 8 || dout.stride(1) % 8 || dout.stride(2) % 8) dout = dout.contiguous();
  fa_check(dout, "dout");
  TORCH_CHECK(lse.is_contiguous() && lse.numel() == B * H * S, "flash_bwd: lse mismatch");
  auto mk = [&](const OptT& given, int64_t heads, const char* n) {
    if (given) {
      fa_check(*given, n);
      TORCH_CHECK(given->size(0) == B && given->size(1) == S && given->size(2) == heads && given->size(3) == D,
                  "flash_bwd: '", n, "' shape mismatch");
      return *given;
    }
    return torch::empty({B, S, heads, D}, q.options());
  };
  Tensor dq = mk(dq_out, H, "dq"), dk = mk(dk_out, Hkv, "dk"), dv = mk(dv_out, Hkv, "dv");
  // -delta' rows | (unused) | 16-byte term rows of -lse log2 e and of -delta' (flash_attn.hip)
  auto delta = torch::empty({10, B, H, S}, q.options().dtype(at::kFloat));
  int64_t st[24];
  const Tensor* ts[8] = {&q, &k, &v, &o, &dout, &dq, &dk, &dv};
  for (int i = 0; i < 8; ++i)
    for (int j = 0; j < 3; ++j) st[3 * i + j] = ts[i]->stride(j);
  check(smdt_flash_bwd(dcode(q), q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), dout.data_ptr(),
                       lse.data_ptr<float>(), delta.data_ptr<float>(), dq.data_ptr(), dk.data_ptr(),
                       dv.data_ptr(), (int)B, (int)H, (int)Hkv, (int)S, (int)D, st, (float)scale,
                       causal ? 1 : 0, (float)dropout_p, (uint64_t)seed, (uint64_t)offset, cur_stream()),
        "flash_bwd");
  return {dq, dk, dv};
}

// ------------------------------------------------------------------ xGMI all-reduce (HIP IPC)
// Raw device pointers cross the Python boundary as int64 (they are IPC mappings, not tensors).
void* vp(int64_t p) { return reinterpret_cast<void*>(static_cast<uintptr_t>(p)); }

int64_t ipc_malloc(int64_t bytes, bool uncached) {
  TORCH_CHECK(bytes > 0, "ipc_malloc: bytes must be positive");
  void* p = nullptr;
  check(smdt_ipc_malloc(bytes, uncached ? 1 : 0, &p), "ipc_malloc");
  return (int64_t)(uintptr_t)p;
}

void ipc_free(int64_t p) { check(smdt_ipc_free(vp(p)), "ipc_free"); }

pybind11::bytes ipc_get_handle(int64_t p) {
  std::string h((size_t)smdt_ipc_handle_bytes(), '\0');
  check(smdt_ipc_get_handle(vp(p), h.data()), "ipc_get_handle");
  return pybind11::bytes(h);
}

int64_t ipc_open(pybind11::bytes handle) {
  const std::string h = handle;
  TORCH_CHECK((int)h.size() == smdt_ipc_handle_bytes(), "ipc_open: handle must be ", smdt_ipc_handle_bytes(), " bytes");
  void* p = nullptr;
  check(smdt_ipc_open(h.data(), &p), "ipc_open");
  return (int64_t)(uintptr_t)p;
}

void ipc_close(int64_t p) { check(smdt_ipc_close(vp(p)), "ipc_close"); }

// One uint32 word of an engine's (uncached) signal buffer as an int32 tensor aliasing device
// memory: the DDP reads the sticky error word back asynchronously (no host sync in the step), and
// tests lower the spin limit to inject a timeout. The tensor does not own the memory.
Tensor signal_word(int64_t sig, int64_t byte_offset) {
  TORCH_CHECK(sig != 0 && byte_offset >= 0 && byte_offset % 4 == 0, "signal_word: bad pointer / offset");
  auto opts = torch::TensorOptions().dtype(torch::kInt32).device(torch::kCUDA, c10::hip::current_device());
  return torch::from_blob(static_cast<char*>(vp(sig)) + byte_offset, {1}, opts);
}

int64_t ar_read_error(int64_t sig) {
  int e = 0;
  check(smdt_ar_read_error(vp(sig), &e), "ar_read_error");
  return e;
}

// out = scale * sum_ranks(in). nranks_local > 1 (loopback tests): in/out are [nranks_local, n]
// and ranks rank .. rank + nranks_local - 1 run in one launch.
void xgmi_allreduce(Tensor in, Tensor out, std::vector<int64_t> data_ptrs, std::vector<int64_t> sig_ptrs,
                    int64_t rank, int64_t nranks_local, int64_t region_bytes, bool two_shot, int64_t blocks,
                    double scale) {
  need_contig(in, "in");
  need_contig(out, "out");
  TORCH_CHECK(in.sizes() == out.sizes() && in.dtype() == out.dtype() && in.device() == out.device(),
              "xgmi_allreduce: in / out mismatch");
  const int world = (int)data_ptrs.size();
  TORCH_CHECK(sig_ptrs.size() == data_ptrs.size() && world >= 2 && world <= smdt_ar_max_ranks(),
              "xgmi_allreduce: need 2..", smdt_ar_max_ranks(), " ranks");
  TORCH_CHECK(blocks >= 1 && blocks <= smdt_ar_max_blocks(), "xgmi_allreduce: blocks out of range");
  int64_t n = in.numel(), stride = 0;
  if (nranks_local > 1) {
    TORCH_CHECK(in.dim() >= 2 && in.size(0) == nranks_local, "xgmi_allreduce loopback: in must be [nranks_local, ...]");
    TORCH_CHECK(blocks * nranks_local <= 512, "xgmi_allreduce loopback: blocks x ranks must stay co-resident (<= 512)");
    n /= nranks_local;
    stride = n;
  }
  std::vector<void*> d(world), s(world);
  for (int r = 0; r < world; ++r) {
    d[r] = vp(data_ptrs[r]);
    s[r] = vp(sig_ptrs[r]);
  }
  TORCH_CHECK(in.is_cuda() && in.device().index() == c10::hip::current_device(),
              "xgmi_allreduce: tensors must live on the current device");
  check(smdt_xgmi_allreduce(dcode(in), in.data_ptr(), out.data_ptr(), stride, n, (float)scale, d.data(), s.data(),
                            world, (int)rank, (int)nranks_local, region_bytes, two_shot ? 1 : 0, (int)blocks,
                            cur_stream()),
        "xgmi_allreduce");
}


// contiguous, bias [N] or None. epi 0: y = x w^T; 1: + bias; 2: h = x w^T + bias, y = gelu(h).
// Returns [y] or [y, h].
// General form: mode 0/1 all-reduce (n = elements), 2 reduce-scatter, 3 all-gather (n = elements
// per slice, slices slice_stride elements apart in the input (RS) / output (AG)). in / out are raw
// views (the reduce-scatter output may alias the input's slice `rank`, the all-gather input may
// alias the output's). Loopback (nranks_local > 1): in / out are [nranks_local, ...] with one row
// per virtual rank. Every element the kernel touches is bounds-checked here against the tensors.
void xgmi_collective(int64_t mode, Tensor in, Tensor out, std::vector<int64_t> data_ptrs, std::vector<int64_t> sig_ptrs,
                     int64_t rank, int64_t nranks_local, int64_t region_bytes, int64_t blocks, int64_t n,
                     int64_t slice_stride, double scale) {
  TORCH_CHECK(mode >= 0 && mode <= 3, "xgmi_collective: mode must be 0..3");
  TORCH_CHECK(in.dtype() == out.dtype() && in.device() == out.device(), "xgmi_collective: in / out mismatch");
  TORCH_CHECK(in.is_cuda() && in.device().index() == c10::hip::current_device(),
              "xgmi_collective: tensors must live on the current device");
  const int world = (int)data_ptrs.size();
  TORCH_CHECK(sig_ptrs.size() == data_ptrs.size() && world >= 2 && world <= smdt_ar_max_ranks(),
              "xgmi_collective: need 2..", smdt_ar_max_ranks(), " ranks");
  TORCH_CHECK(blocks >= 1 && blocks <= smdt_ar_max_blocks(), "xgmi_collective: blocks out of range");
  TORCH_CHECK(n > 0, "xgmi_collective: empty message");
  int64_t in_per = in.numel(), out_per = out.numel(), in_rs = 0, out_rs = 0;
  if (nranks_local > 1) {
    TORCH_CHECK(in.dim() == 2 && out.dim() == 2 && in.size(0) == nranks_local && out.size(0) == nranks_local &&
                    in.stride(1) == 1 && out.stride(1) == 1,
                "xgmi_collective loopback: in / out must be [nranks_local, m] with unit inner stride");
    TORCH_CHECK(blocks * nranks_local <= 512, "xgmi_collective loopback: blocks x ranks must stay co-resident (<= 512)");
    in_per = in.size(1);
    out_per = out.size(1);
    in_rs = in.stride(0);
    out_rs = out.stride(0);
  } else {
    TORCH_CHECK(in.is_contiguous() && out.is_contiguous(), "xgmi_collective: contiguous tensors");
  }
  const int64_t span = (int64_t)(world - 1) * slice_stride + n;
  const int64_t need_in = mode == 2 ? span : n, need_out = mode == 3 ? span : n;
  TORCH_CHECK(in_per >= need_in && out_per >= need_out, "xgmi_collective: tensors too small for n = ", n,
              ", slice stride ", slice_stride);
  std::vector<void*> d(world), s(world);
  for (int r = 0; r < world; ++r) {
    d[r] = vp(data_ptrs[r]);
    s[r] = vp(sig_ptrs[r]);
  }
  check(smdt_xgmi_collective((int)mode, dcode(in), in.data_ptr(), out.data_ptr(), in_rs, out_rs, n, slice_stride,
                             (float)scale, d.data(), s.data(), world, (int)rank, (int)nranks_local, region_bytes,
                             (int)blocks, cur_stream()),
        "xgmi_collective");
}

int64_t relay_read_error(int64_t sig) {
  int e = 0;
  check(smdt_relay_read_error(vp(sig), &e), "relay_read_error");
  return e;
}

// Pairwise TP exchange over all xGMI links (xgmi_relay.hip): out (on this rank) = in of the
// partner. Loopback (nranks_local > 1): in / out are [nranks_local, m] rows, one per virtual rank.
void xgmi_relay(Tensor in, Tensor out, std::vector<int64_t> stage_ptrs, std::vector<int64_t> sig_ptrs,
                std::vector<int64_t> partners, int64_t rank, int64_t nranks_local, int64_t slot_bytes, int64_t sub,
                int64_t epoch, bool dev_epoch) {
  TORCH_CHECK(in.dtype() == out.dtype() && in.device() == out.device(), "xgmi_relay: in / out mismatch");
  TORCH_CHECK(in.is_cuda() && in.device().index() == c10::hip::current_device(),
              "xgmi_relay: tensors must live on the current device");
  TORCH_CHECK(in.scalar_type() == at::kFloat || in.scalar_type() == at::kBFloat16 || in.scalar_type() == at::kHalf,
              "xgmi_relay: fp32 / bf16 / fp16");
  const int world = (int)stage_ptrs.size();
  TORCH_CHECK(sig_ptrs.size() == stage_ptrs.size() && partners.size() == stage_ptrs.size() &&
                  (world == 2 || world == 4 || world == 8),
              "xgmi_relay: 2, 4 or 8 ranks");
  TORCH_CHECK(sub >= 1 && sub <= smdt_relay_max_sub(), "xgmi_relay: sub out of range");
  TORCH_CHECK(epoch >= 1 && epoch <= 0xffffffffll, "xgmi_relay: epoch must be a positive uint32");
  int64_t n = in.numel(), in_rs = 0, out_rs = 0;
  if (nranks_local > 1) {
    TORCH_CHECK(in.dim() == 2 && out.dim() == 2 && in.size(0) == nranks_local && out.size(0) == nranks_local &&
                    in.stride(1) == 1 && out.stride(1) == 1 && out.size(1) == in.size(1),
                "xgmi_relay loopback: in / out must be [nranks_local, m] with unit inner stride");
    TORCH_CHECK(2 * sub * world * nranks_local <= 512, "xgmi_relay loopback: blocks must stay co-resident (<= 512)");
    n = in.size(1);
    in_rs = in.stride(0);
    out_rs = out.stride(0);
  } else {
    TORCH_CHECK(in.is_contiguous() && out.is_contiguous() && out.numel() == n, "xgmi_relay: contiguous, equal sizes");
  }
  std::vector<void*> d(world), s(world);
  std::vector<int> p(world);
  for (int r = 0; r < world; ++r) {
    d[r] = vp(stage_ptrs[r]);
    s[r] = vp(sig_ptrs[r]);
    p[r] = (int)partners[r];
  }
  check(smdt_xgmi_relay(dcode(in), in.data_ptr(), out.data_ptr(), in_rs, out_rs, n, d.data(), s.data(), p.data(), world,
                        (int)rank, (int)nranks_local, slot_bytes, (int)sub, (uint32_t)epoch, dev_epoch ? 1 : 0,
                        cur_stream()),
        "xgmi_relay");
}

void relay_reset(int64_t sig) { check(smdt_relay_reset(vp(sig), cur_stream()), "relay_reset"); }

// Device epochs (xgmi_relay.hip): advance the local ranks' call counters by n on the current stream.
void relay_epoch_bump(std::vector<int64_t> sig_ptrs, int64_t rank, int64_t nranks_local, int64_t n) {
  std::vector<void*> s(sig_ptrs.size());
  for (size_t r = 0; r < sig_ptrs.size(); ++r) s[r] = vp(sig_ptrs[r]);
  TORCH_CHECK(n >= 1 && n <= 0xffffll, "relay_epoch_bump: n out of range");
  check(smdt_relay_epoch_bump(s.data(), (int)s.size(), (int)rank, (int)nranks_local, (uint32_t)n, cur_stream()),
        "relay_epoch_bump");
}

}  // namespace

void register_blaslt(pybind11::module_& m);

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "smdt_amd gfx950 (MI355X) HIP kernel library";
  register_blaslt(m);
  using pybind11::arg;
  m.def("layernorm_fwd", &layernorm_fwd, arg("x"), arg("res"), arg("bias"), arg("gamma"), arg("beta"),
        arg("eps"), arg("p_drop"), arg("seed"), arg("offset"), arg("rms"), arg("want_s"),
        arg("out_y") = pybind11::none(), arg("x2") = pybind11::none());
  m.def("layernorm_bwd", &layernorm_bwd, arg("dy"), arg("ds_in"), arg("s"), arg("gamma"), arg("mean"),
        arg("rstd"), arg("p_drop"), arg("seed"), arg("offset"), arg("rms"), arg("want_dx"), arg("want_dbias"),
        arg("dgamma_acc") = pybind11::none(), arg("dbeta_acc") = pybind11::none(),
        arg("dbias_acc") = pybind11::none(), arg("out_dx") = pybind11::none(), arg("dy2") = pybind11::none());
  m.def("bias_act_fwd", &bias_act_fwd);
  m.def("bias_act_bwd", &bias_act_bwd, arg("dy"), arg("x"), arg("bias"), arg("act"), arg("want_dbias"),
        arg("dbias_acc") = pybind11::none());
  m.def("swiglu_fwd", &swiglu_fwd);
  m.def("swiglu_bwd", &swiglu_bwd);
  m.def("softmax_fwd", &softmax_fwd);
  m.def("softmax_bwd", &softmax_bwd);
  m.def("adam", &adam);
  m.def("sumsq", &sumsq);
  m.def("clip_coef", &clip_coef);
  m.def("scale_", &scale_);
  m.def("cast_", &cast_);
  m.def("rope_", &rope_);
  m.def("transpose2d", &transpose2d);
  m.def("paced_copy", &paced_copy);
  m.def("gather_rows", &gather_rows);
  m.def("aug_depthwise", &aug_depthwise);
  m.def("aug_median3", &aug_median3);
  m.def("bias_grad", &bias_grad);
  m.def("gemm_tn_supported", &gemm_tn_supported, arg("a"), arg("b"));
  m.def("gemm_tn", &gemm_tn, arg("a"), arg("b"), arg("epi") = 0, arg("bias") = pybind11::none(),
        arg("out") = pybind11::none(), arg("out2") = pybind11::none(), arg("max_blocks") = 0,
        arg("var") = 0, arg("aux") = pybind11::none());
  m.def("wgrad_mfma", &wgrad_mfma, arg("main_grad"), arg("dy"), arg("x"), arg("max_splits") = 0);
  m.def("wgrad_grouped", &wgrad_grouped, arg("main_grads"), arg("dys"), arg("xs"),
        arg("biases") = std::vector<Tensor>{}, arg("overwrite") = std::vector<bool>{}, arg("cus") = 0);
  m.def("ce_stats", &ce_stats);
  m.def("set_rng_step", &set_rng_step);
  m.def("adam_capturable", &adam_capturable);
  m.def("ce_fused_local", &ce_fused_local);
  m.def("ce_bwd", &ce_bwd);
  m.def("ce_fused", &ce_fused);
  namespace py = pybind11;
  m.def("flash_fwd", &flash_fwd, py::arg("q"), py::arg("k"), py::arg("v"), py::arg("scale"), py::arg("causal"),
        py::arg("out") = py::none(), py::arg("dropout_p") = 0.0, py::arg("seed") = 0, py::arg("offset") = 0);
  m.def("ipc_malloc", &ipc_malloc, py::arg("bytes"), py::arg("uncached"));
  m.def("ipc_free", &ipc_free);
  m.def("ipc_get_handle", &ipc_get_handle);
  m.def("ipc_open", &ipc_open);
  m.def("ipc_close", &ipc_close);
  m.def("ar_read_error", &ar_read_error);
  m.def("signal_word", &signal_word, py::arg("sig"), py::arg("byte_offset"));
  m.def("ar_word_offset", &smdt_ar_word_offset);
  m.def("relay_word_offset", &smdt_relay_word_offset);
  m.def("ar_signal_bytes", &smdt_ar_signal_bytes);
  m.def("ar_max_blocks", &smdt_ar_max_blocks);
  m.def("xgmi_allreduce", &xgmi_allreduce, py::arg("input"), py::arg("out"), py::arg("data_ptrs"), py::arg("sig_ptrs"),
        py::arg("rank"), py::arg("nranks_local"), py::arg("region_bytes"), py::arg("two_shot"), py::arg("blocks"),
        py::arg("scale") = 1.0);
  m.def("xgmi_collective", &xgmi_collective, py::arg("mode"), py::arg("input"), py::arg("out"), py::arg("data_ptrs"),
        py::arg("sig_ptrs"), py::arg("rank"), py::arg("nranks_local"), py::arg("region_bytes"), py::arg("blocks"),
        py::arg("n"), py::arg("slice_stride"), py::arg("scale") = 1.0);
  m.def("xgmi_relay", &xgmi_relay, py::arg("input"), py::arg("out"), py::arg("stage_ptrs"), py::arg("sig_ptrs"),
        py::arg("partners"), py::arg("rank"), py::arg("nranks_local"), py::arg("slot_bytes"), py::arg("sub"),
        py::arg("epoch"), py::arg("dev_epoch") = false);
  m.def("relay_reset", &relay_reset, py::arg("sig"));
  m.def("relay_epoch_bump", &relay_epoch_bump, py::arg("sig_ptrs"), py::arg("rank"), py::arg("nranks_local"),
        py::arg("n"));
  m.def("relay_signal_bytes", &smdt_relay_signal_bytes);
  m.def("relay_read_error", &relay_read_error);
  m.def("flash_bwd", &flash_bwd, py::arg("q"), py::arg("k"), py::arg("v"), py::arg("o"), py::arg("dout"),
        py::arg("lse"), py::arg("scale"), py::arg("causal"), py::arg("dq") = py::none(), py::arg("dk") = py::none(),
        py::arg("dv") = py::none(), py::arg("dropout_p") = 0.0, py::arg("seed") = 0, py::arg("offset") = 0);
}
