"""Shared numerics for the kernel tests: inputs that make every term of a gradient visible, a
row-relative error criterion, and fp32 references with a knob that mutates the softmax term.

The GPU tests (``test_kernels_gpu.py``) judge the HIP kernels against these references; the CPU
test ``test_numerics_sensitivity.py`` proves each criterion can fail: an emulation of the kernel's
16-bit rounding points passes it, while the same reference with the softmax term dropped
(``soft=0``) or scaled by 1.1 (``soft=1.1``), an all-zero output, or a gradient zeroed past row 64
is rejected. A check that a wrong kernel can pass is no check.
"""
import torch

# Row-relative tolerances used by the GPU tests (sized from the CPU sensitivity test: the bf16
# emulations land at <= 0.8 % of the row max, every mutation at >= 6 %).
CE_TOL = 0.03
SOFTMAX_TOL = 0.03


def row_rel_err(out, ref, floor_frac: float = 1e-4, row_floor=None) -> float:
    """max over rows of max|out - ref| / max|ref| (rows = every index but the last). Rows whose
    reference is ~0 are judged against ``floor_frac`` of the global max instead; ``row_floor``
    (one value per row) raises a row's denominator to the error its 16-bit inputs alone imply."""
    o = out.detach().float().reshape(-1, out.shape[-1])
    r = ref.detach().float().reshape(-1, ref.shape[-1]).to(o.device)
    den = r.abs().amax(-1).clamp_min(floor_frac * r.abs().max().clamp_min(1e-30))
    if row_floor is not None:
        den = torch.maximum(den, row_floor.detach().float().reshape(-1).to(o.device))
    return ((o - r).abs().amax(-1) / den).max().item()


def softmax_grad_floor(y, dy, scale):
    """Per-row magnitude of the error a 16-bit stored y alone puts into scale * y (dy - sum(dy y)):
    a few 2^-8 * scale * max|dy| * max y (y_i + y_j != 1 after rounding). Rows of a peaked softmax
    cancel down to that level."""
    return 2.0 ** -6 * scale * dy.float().abs().amax(-1) * y.float().amax(-1)


def assert_rows_close(out, ref, tol, what="", row_floor=None):
    e = row_rel_err(out, ref, row_floor=row_floor)
    assert e <= tol, f"{what}: row-relative error {e:.4g} > {tol}"


# ------------------------------------------------------------------------------ cross entropy

def ce_case(N, V, vocab=0, device="cpu", seed=9, scale=8.0):
    """Peaked bf16 logits (std ``scale``) so softmax mass sits on a few columns; half the targets
    are the row's argmax, half are random columns (the softmax term then dominates), one row is
    ignored (-100). O(1) signed per-row dloss."""
    g = torch.Generator().manual_seed(seed)
    nv = vocab or V
    logits = (scale * torch.randn(N, V, generator=g)).bfloat16()
    tgt = torch.randint(0, nv, (N,), generator=g)
    am = logits[:, :nv].float().argmax(-1)
    tgt[::2] = am[::2]
    tgt[5] = -100
    dl = torch.randn(N, generator=g)
    return logits.to(device), tgt.to(device), dl.to(device)


def ce_ref(logits, tgt, dl, vocab=0, soft=1.0):
    """fp32 per-token CE loss and d(sum dl * loss)/dlogits with the softmax term scaled by
    ``soft`` (1 = correct). Columns >= vocab (if > 0) are padding: no mass, zero gradient."""
    z = logits.float()
    V = z.shape[-1]
    nv = vocab or V
    zz = z[:, :nv]
    lse = torch.logsumexp(zz, -1)
    valid = tgt >= 0
    t = tgt.clamp_min(0)
    loss = torch.where(valid, lse - zz.gather(1, t[:, None])[:, 0], torch.zeros_like(lse))
    p = torch.softmax(zz, -1)
    grad = torch.zeros_like(z)
    grad[:, :nv] = soft * p
    grad[torch.arange(z.shape[0], device=z.device), t] -= 1.0
    grad = grad * (dl * valid)[:, None]
    return loss, grad


def ce_kernel_emulation(logits, tgt, dl, vocab=0):
    """The CE kernels' rounding: fp32 math, dlogits stored in the logits' 16-bit type."""
    loss, grad = ce_ref(logits, tgt, dl, vocab)
    return loss, grad.to(logits.dtype)


# ---------------------------------------------------------------------- LM head + CE (TP = 1)

def lmce_case(s=96, b=3, H=256, V=50304, vocab=0, device="cpu", seed=12):
    """h ~ N(0, 1), W ~ N(0, 0.25^2): logits with std ~4 (peaked); targets half argmax, half
    random, one ignored; O(1) signed dloss."""
    g = torch.Generator().manual_seed(seed)
    nv = vocab or V
    h = torch.randn(s, b, H, generator=g).bfloat16()
    w = (0.25 * torch.randn(V, H, generator=g)).bfloat16()
    lg = (h.float().reshape(-1, H) @ w.float().t())[:, :nv]
    tgt = torch.randint(0, nv, (s * b,), generator=g)
    tgt[::2] = lg.argmax(-1)[::2]
    tgt[3 * b + 1] = -100
    dl = torch.randn(s, b, generator=g)
    return h.to(device), w.to(device), tgt.view(s, b).to(device), dl.to(device)


def lmce_ref(h, w, logits16, tgt, dl, vocab=0, soft=1.0):
    """fp32 loss / dh / dW of sum(dl * CE(h W^T)) given the 16-bit logits the kernel's GEMM made
    (so the check isolates the CE + backward GEMMs from the forward GEMM's output rounding)."""
    H = h.shape[-1]
    loss, G = ce_ref(logits16.reshape(-1, logits16.shape[-1]), tgt.reshape(-1), dl.reshape(-1).float(), vocab, soft)
    dh = (G @ w.float()).view(h.shape)
    dw = G.t() @ h.float().reshape(-1, H)
    return loss.view(tgt.shape), dh, dw


def lmce_kernel_emulation(h, w, logits16, tgt, dl, vocab=0):
    """LMHeadCrossEntropy's rounding points: D = softmax - onehot stored 16-bit in place; dX = D W
    in 16-bit then scaled by dl in 16-bit; dW = D^T (h * dl rounded to 16-bit), fp32 accumulate."""
    H = h.shape[-1]
    loss, D = ce_ref(logits16.reshape(-1, logits16.shape[-1]), tgt.reshape(-1),
                     torch.ones(tgt.numel(), device=h.device), vocab)
    D = D.to(h.dtype).float()
    d = dl.reshape(-1, 1).float()
    dh = ((D @ w.float()).to(h.dtype).float() * d).to(h.dtype).view(h.shape)
    hs = (h.float().reshape(-1, H) * d).to(h.dtype).float()
    dw = D.t() @ hs
    return loss.view(tgt.shape), dh, dw


# ----------------------------------------------------------------------------------- softmax

def softmax_case(sk, causal, b=2, np_=4, device="cpu", seed=5, std=8.0):
    """Sharp scores: x ~ N(0, std^2) with scale 0.125 -> scaled std 1 (not near-uniform rows)."""
    g = torch.Generator().manual_seed(seed)
    x = (std * torch.randn(b, np_, sk, sk, generator=g)).bfloat16()
    dy = torch.randn(b, np_, sk, sk, generator=g).bfloat16()
    return x.to(device), dy.to(device)


def softmax_ref(x, dy, scale, causal, mask=None):
    xr = x.detach().float().requires_grad_()
    s = xr * scale
    sk = x.shape[-1]
    if causal:
        s = s.masked_fill(torch.ones(x.shape[-2], sk, device=x.device, dtype=torch.bool).triu(1), float("-inf"))
    elif mask is not None:
        s = s.masked_fill(mask, float("-inf"))
    y = torch.softmax(s, -1)
    y.backward(dy.float())
    return y.detach(), xr.grad


def vp_lmce_two_shards(h, w, tgt, dl, vocab=0, ranks=2, local_pass=None):
    """The vocab-parallel LM-head CE math of ``VocabParallelLMHeadCE`` run for ``ranks`` vocab
    shards in one process: per shard the logits GEMM and ``local_pass`` (the HIP kernel or its CPU
    reference), the statistics combined, the one-hot subtracted at one element per row, and the
    backward products with the per-row scale c dl on the hidden side. Returns (loss, dh, dW,
    16-bit logits of all shards) for comparison with ``lmce_ref`` on the same logits."""
    from smdt_amd.parallel import tensor_parallel as tp
    local_pass = local_pass or tp.ce_local_pass
    H = h.shape[-1]
    V = w.shape[0]
    vl = V // ranks
    x = h.reshape(-1, H)
    t = tgt.reshape(-1)
    shards, stats, lgs = [], [], []
    for r in range(ranks):
        ws_ = w[r * vl:(r + 1) * vl]
        lg = x @ ws_.t() if not x.is_cuda else tp.linear_rows(x, ws_)
        lg = lg.to(h.dtype)
        lgs.append(lg.clone())
        vv = min(max(vocab - r * vl, 0), vl) if vocab else 0
        vv = 0 if vv == vl else vv
        st = local_pass(lg, t, r * vl, vv)
        shards.append((lg, vv))
        stats.append(st)
    allst = torch.stack(stats)
    d = dl.reshape(-1).float()
    dh = torch.zeros(x.shape, dtype=torch.float32, device=x.device)
    dws = []
    for r, (e, vv) in enumerate(shards):
        loss, c = tp.combine_ce_stats(allst, stats[r], t, -100)
        tp.subtract_onehot_(e, t, c, r * vl, vv, -100)
        rr = (d * c)[:, None]
        dh += (e.float() @ w[r * vl:(r + 1) * vl].float()) * rr
        dws.append(e.float().t() @ (x.float() * rr).to(h.dtype).float())
    return loss.view(tgt.shape), dh.view(h.shape), torch.cat(dws), torch.cat(lgs, -1)
