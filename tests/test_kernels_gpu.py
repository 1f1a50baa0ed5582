"""Numerics of every gfx950 HIP kernel against a plain PyTorch fp32 reference of the same op.

All tests need the MI355X and the in-tree ``smdt_amd/_C.so`` (they fail loudly if it cannot
load: the GPU path never falls back to eager PyTorch).
"""
import math

import pytest
import torch
import torch.nn.functional as F

from smdt_amd.ops import _ext
from smdt_amd.ops import functional as SF

import _numerics as N

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _C():
    return _ext.ext()


def test_extension_loaded_from_tree():
    C = _C()
    import os
    import smdt_amd
    assert os.path.dirname(os.path.realpath(C.__file__)) == os.path.dirname(os.path.realpath(smdt_amd.__file__))


@pytest.mark.parametrize("H", [768, 1024, 4096])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("rms", [False, True])
def test_layernorm_fwd_bwd(H, dtype, rms):
    torch.manual_seed(0)
    rows = 333
    x = torch.randn(rows, H, device=DEV, dtype=dtype, requires_grad=True)
    g = (1 + 0.1 * torch.randn(H, device=DEV, dtype=dtype)).requires_grad_()
    b = (0.1 * torch.randn(H, device=DEV, dtype=dtype)).requires_grad_() if not rms else None
    y, s = SF.bias_dropout_add_norm(x, None, None, g, b, 0.0, False, 1e-5, rms)
    xr = x.detach().float().requires_grad_()
    gr = g.detach().float().requires_grad_()
    br = b.detach().float().requires_grad_() if b is not None else None
    if rms:
        yr = xr * torch.rsqrt(xr.pow(2).mean(-1, keepdim=True) + 1e-5) * gr
    else:
        yr = F.layer_norm(xr, (H,), gr, br, 1e-5)
    tol = 2e-2 if dtype == torch.bfloat16 else 1e-4
    torch.testing.assert_close(y.float(), yr, atol=tol, rtol=tol)
    dy = torch.randn_like(y)
    y.backward(dy)
    yr.backward(dy.float())
    torch.testing.assert_close(x.grad.float(), xr.grad, atol=5 * tol, rtol=5 * tol)
    torch.testing.assert_close(g.grad.float(), gr.grad, atol=tol * math.sqrt(rows) * 4, rtol=5 * tol)
    if b is not None:
        torch.testing.assert_close(b.grad.float(), br.grad, atol=tol * math.sqrt(rows) * 4, rtol=5 * tol)


def test_fused_bias_residual_layernorm():
    torch.manual_seed(1)
    rows, H = 512, 1024
    dt = torch.bfloat16
    x = torch.randn(rows, H, device=DEV, dtype=dt, requires_grad=True)
    res = torch.randn(rows, H, device=DEV, dtype=dt, requires_grad=True)
    bias = (0.1 * torch.randn(H, device=DEV, dtype=dt)).requires_grad_()
    g = (1 + 0.1 * torch.randn(H, device=DEV, dtype=dt)).requires_grad_()
    be = (0.1 * torch.randn(H, device=DEV, dtype=dt)).requires_grad_()
    y, s = SF.bias_dropout_add_norm(x, bias, res, g, be, 0.0, True, 1e-5, False)
    leaves = [x, res, bias, g, be]
    ref = [t.detach().float().requires_grad_() for t in leaves]
    sr = ref[1] + (ref[0] + ref[2])
    yr = F.layer_norm(sr, (H,), ref[3], ref[4], 1e-5)
    torch.testing.assert_close(s.float(), sr, atol=3e-2, rtol=2e-2)
    torch.testing.assert_close(y.float(), yr, atol=5e-2, rtol=3e-2)
    dy, ds = torch.randn_like(y), torch.randn_like(s)
    torch.autograd.backward([y, s], [dy, ds])
    torch.autograd.backward([yr, sr], [dy.float(), ds.float()])
    for a, r in zip(leaves, ref):
        torch.testing.assert_close(a.grad.float(), r.grad, atol=0.5, rtol=5e-2)


def test_fused_norm_with_pending_summand():
    """A row-parallel output whose reduce-scatter combine was left to the norm (``x._smdt_add`` =
    the peer's partial, tensor_parallel.defer_rs_add): the kernel reads both summands, s = res +
    (x + x2 + bias), and x's gradient is that of x + x2. fp32 reference of the same op."""
    torch.manual_seed(3)
    rows, H = 512, 1024
    dt = torch.bfloat16
    x = torch.randn(rows, H, device=DEV, dtype=dt, requires_grad=True)
    x2 = torch.randn(rows, H, device=DEV, dtype=dt)
    res = torch.randn(rows, H, device=DEV, dtype=dt, requires_grad=True)
    bias = (0.1 * torch.randn(H, device=DEV, dtype=dt)).requires_grad_()
    g = (1 + 0.1 * torch.randn(H, device=DEV, dtype=dt)).requires_grad_()
    be = (0.1 * torch.randn(H, device=DEV, dtype=dt)).requires_grad_()
    x._smdt_add = x2
    y, s = SF.bias_dropout_add_norm(x, bias, res, g, be, 0.0, True, 1e-5, False)
    assert not hasattr(x, "_smdt_add")          # consumed
    leaves = [x, res, bias, g, be]
    ref = [t.detach().float().requires_grad_() for t in leaves]
    sr = ref[1] + (ref[0] + x2.float() + ref[2])
    yr = F.layer_norm(sr, (H,), ref[3], ref[4], 1e-5)
    torch.testing.assert_close(s.float(), sr, atol=3e-2, rtol=2e-2)
    torch.testing.assert_close(y.float(), yr, atol=5e-2, rtol=3e-2)
    dy, ds = torch.randn_like(y), torch.randn_like(s)
    torch.autograd.backward([y, s], [dy, ds])
    torch.autograd.backward([yr, sr], [dy.float(), ds.float()])
    for a, r in zip(leaves, ref):
        torch.testing.assert_close(a.grad.float(), r.grad, atol=0.5, rtol=5e-2)
    # without the summand the output differs by far more than the tolerance (the test can fail)
    y0, _ = SF.bias_dropout_add_norm(x.detach(), bias.detach(), res.detach(), g.detach(), be.detach(),
                                     0.0, True, 1e-5, False)
    assert (y0.float() - yr).abs().max() > 0.5


def test_fused_dropout_mask_consistency():
    torch.manual_seed(2)
    rows, H, p = 256, 1024, 0.25
    dt = torch.bfloat16
    x = torch.randn(rows, H, device=DEV, dtype=dt, requires_grad=True)
    res = torch.zeros(rows, H, device=DEV, dtype=dt)
    g = torch.ones(H, device=DEV, dtype=dt, requires_grad=True)
    be = torch.zeros(H, device=DEV, dtype=dt, requires_grad=True)
    y, s = SF.bias_dropout_add_norm(x, None, res, g, be, p, True, 1e-5, False)
    kept = (s != 0)
    frac = kept.float().mean().item()
    assert abs(frac - (1 - p)) < 0.02
    torch.testing.assert_close(s[kept].float(), (x.detach()[kept].float() / (1 - p)), atol=2e-2, rtol=1e-2)
    s.backward(torch.ones_like(s))
    # ds = 1 everywhere -> dx = mask / (1 - p): zero exactly where dropped
    assert torch.all(x.grad[~kept] == 0)
    torch.testing.assert_close(x.grad[kept].float(), torch.full_like(x.grad[kept].float(), 1 / (1 - p)),
                               atol=1e-2, rtol=1e-2)


@pytest.mark.parametrize("approx", ["tanh", "none"])
def test_bias_gelu(approx):
    torch.manual_seed(3)
    x = torch.randn(1000, 4096, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    b = torch.randn(4096, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    y = SF.bias_gelu(x, b, approx)
    xr, br = x.detach().float().requires_grad_(), b.detach().float().requires_grad_()
    yr = F.gelu(xr + br, approximate=approx)
    torch.testing.assert_close(y.float(), yr, atol=2e-2, rtol=2e-2)
    dy = torch.randn_like(y)
    y.backward(dy)
    yr.backward(dy.float())
    torch.testing.assert_close(x.grad.float(), xr.grad, atol=3e-2, rtol=3e-2)
    torch.testing.assert_close(b.grad.float(), br.grad, atol=1.0, rtol=2e-2)


@pytest.mark.parametrize("rows,N", [(1001, 4096), (300_001, 64), (4, 2048)])
def test_bias_gelu_partial_free_launch_shapes(rows, N):
    """The partial-free launches (forward, and backward without d(bias)) give each thread one
    4-row batch; row counts not a multiple of 4 and past grid.y's 65535 slices (the slice then
    loops over more rows) still cover every row exactly once."""
    torch.manual_seed(5)
    x = torch.randn(rows, N, device=DEV, dtype=torch.bfloat16)
    b = torch.randn(N, device=DEV, dtype=torch.bfloat16)
    dy = torch.randn_like(x)
    z = x.float() + b.float()
    y = _C().bias_act_fwd(x, b, 0)
    torch.testing.assert_close(y.float(), F.gelu(z, approximate="tanh"), atol=2e-2, rtol=2e-2)
    dx, _ = _C().bias_act_bwd(dy, x, b, 0, False, None)
    zr = z.clone().requires_grad_()
    F.gelu(zr, approximate="tanh").backward(dy.float())
    torch.testing.assert_close(dx.float(), zr.grad, atol=3e-2, rtol=3e-2)


@pytest.mark.parametrize("rows,ffn", [(777, 1024), (70_001, 64)])
def test_swiglu(rows, ffn):
    """[rows, 2F] -> [rows, F]; 70,001 rows exercise the row stride past grid.y's 65,535."""
    torch.manual_seed(4)
    x = torch.randn(rows, 2 * ffn, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    y = SF.swiglu(x)
    xr = x.detach().float().requires_grad_()
    g, u = xr.chunk(2, -1)
    yr = F.silu(g) * u
    torch.testing.assert_close(y.float(), yr, atol=3e-2, rtol=2e-2)
    dy = torch.randn_like(y)
    y.backward(dy)
    yr.backward(dy.float())
    torch.testing.assert_close(x.grad.float(), xr.grad, atol=5e-2, rtol=3e-2)


@pytest.mark.parametrize("sk", [128, 1024, 2048])
@pytest.mark.parametrize("causal", [True, False])
def test_scaled_masked_softmax(sk, causal):
    """Sharp scores (scaled std 1), judged per row relative to the row's max (tests/_numerics.py).
    Mutation check (tests/test_numerics_sensitivity.py): an all-zero y or dx, dx x1.1, or dx zero
    past row 64 fail this criterion (row-relative errors 1.0 / 1.0 / 0.10 / 1.0 vs tol 0.03); a bf16
    emulation of the kernel passes at <= 0.01."""
    x, dy = N.softmax_case(sk, causal, device=DEV)
    x.requires_grad_()
    y = SF.scaled_masked_softmax(x, None, 0.125, causal)
    yr, dxr = N.softmax_ref(x, dy, 0.125, causal)
    N.assert_rows_close(y, yr, N.SOFTMAX_TOL, "y")
    y.backward(dy)
    N.assert_rows_close(x.grad, dxr, N.SOFTMAX_TOL, "dx", row_floor=N.softmax_grad_floor(yr, dy, 0.125))


def test_softmax_explicit_mask():
    """Arbitrary [b, 1, sq, sk] mask, forward and backward, row-relative (an unmasked softmax or
    dx x1.1 fails the criterion: tests/test_numerics_sensitivity.py)."""
    g = torch.Generator().manual_seed(6)
    x = (8 * torch.randn(2, 3, 64, 256, generator=g)).bfloat16().to(DEV).requires_grad_()
    mask = (torch.rand(2, 1, 64, 256, generator=g) < 0.3).to(DEV)
    dy = torch.randn(2, 3, 64, 256, generator=g).bfloat16().to(DEV)
    y = SF.scaled_masked_softmax(x, mask, 0.125, False)
    yr, dxr = N.softmax_ref(x, dy, 0.125, False, mask)
    N.assert_rows_close(y, yr, N.SOFTMAX_TOL, "y")
    assert torch.all(y[mask.expand_as(y)] == 0)
    y.backward(dy)
    N.assert_rows_close(x.grad, dxr, N.SOFTMAX_TOL, "dx", row_floor=N.softmax_grad_floor(yr, dy, 0.125))


def test_fused_adam_matches_reference():
    torch.manual_seed(7)
    n = 1_000_003
    p = torch.randn(n, device=DEV)
    g = torch.randn(n, device=DEV)
    m = torch.zeros(n, device=DEV)
    v = torch.zeros(n, device=DEV)
    model = torch.empty(n, device=DEV, dtype=torch.bfloat16)
    pr, mr, vr = p.clone(), m.clone(), v.clone()
    lr, b1, b2, eps, wd = 1e-3, 0.9, 0.95, 1e-8, 0.1
    mul = torch.tensor([0.5], device=DEV)
    for step in (1, 2, 3):
        _C().adam(p, g, m, v, model, lr, b1, b2, eps, wd, step, True, mul, None)
        gg = g * 0.5
        mr.mul_(b1).add_(gg, alpha=1 - b1)
        vr.mul_(b2).addcmul_(gg, gg, value=1 - b2)
        denom = (vr.sqrt() / math.sqrt(1 - b2 ** step)) + eps
        pr.mul_(1 - lr * wd)
        pr.addcdiv_(mr, denom, value=-lr / (1 - b1 ** step))
    torch.testing.assert_close(p, pr, atol=1e-6, rtol=1e-5)
    torch.testing.assert_close(model.float(), pr, atol=1e-2, rtol=1e-2)
    found = torch.ones(1, device=DEV, dtype=torch.int32)
    before = p.clone()
    _C().adam(p, g, m, v, model, lr, b1, b2, eps, wd, 4, True, mul, found)
    assert torch.equal(p, before), "found_inf must skip the step"


def test_sumsq_and_inf_detection():
    x = torch.randn(3_000_001, device=DEV)
    found = torch.zeros(1, device=DEV, dtype=torch.int32)
    s = _C().sumsq(x, found)
    torch.testing.assert_close(s, (x.double() ** 2).sum().float().view(1), rtol=1e-4, atol=1e-2)
    assert found.item() == 0
    x[12345] = float("inf")
    _C().sumsq(x, found)
    assert found.item() == 1
    xb = torch.randn(100_000, device=DEV, dtype=torch.bfloat16)
    sb = _C().sumsq(xb, None)
    torch.testing.assert_close(sb, (xb.double() ** 2).sum().float().view(1), rtol=1e-3, atol=1e-2)


@pytest.mark.parametrize("nh", [4, 16])
def test_rope_inplace_and_inverse(nh):
    """nh 4: the grid-stride kernel; nh 16 (>= 64 8-pair groups per token): the token-per-block
    kernel; both also on a strided [tokens, heads, d] view of a wider fused-QKV row."""
    torch.manual_seed(8)
    s, b, d = 64, 3, 128
    x = torch.randn(s * b, nh, d, device=DEV, dtype=torch.bfloat16)
    cos, sin = SF.rope_tables(s, d, device=DEV)
    y = x.clone()
    _C().rope_(y, cos, sin, d, b, s, False)
    pos = torch.arange(s * b, device=DEV) // b
    yr = SF._rope_ref(x, cos, sin, d, pos)
    torch.testing.assert_close(y.float(), yr.float(), atol=2e-2, rtol=2e-2)
    _C().rope_(y, cos, sin, d, b, s, True)
    torch.testing.assert_close(y.float(), x.float(), atol=3e-2, rtol=3e-2)
    wide = torch.randn(s * b, (nh + 2) * d, device=DEV, dtype=torch.bfloat16)   # [q | k | v]-like row
    keep = wide.clone()
    view = wide[:, : nh * d].view(s * b, nh, d)
    _C().rope_(view, cos, sin, d, b, s, False)
    ref = SF._rope_ref(keep[:, : nh * d].view(s * b, nh, d), cos, sin, d, pos)
    torch.testing.assert_close(view.float(), ref.float(), atol=2e-2, rtol=2e-2)
    assert torch.equal(wide[:, nh * d:], keep[:, nh * d:])                 # the rest of the row untouched


@pytest.mark.parametrize("V", [50304, 1000])
def test_cross_entropy(V):
    """Peaked logits (std 8), half the targets the row's argmax and half random, O(1) signed
    dloss; gradient judged per row relative to the row max. Mutation check
    (tests/test_numerics_sensitivity.py): dropping the softmax term or scaling it by 1.1 / 0.9
    gives row-relative errors >= 300 vs tol 0.03; a bf16 emulation of the kernel gives 0.004."""
    logits, tgt, dl = N.ce_case(300, V, device=DEV)
    logits.requires_grad_()
    loss = SF.cross_entropy(logits, tgt)
    ref, gref = N.ce_ref(logits, tgt, dl)
    torch.testing.assert_close(loss, ref, atol=5e-3, rtol=1e-3)
    (loss * dl).sum().backward()
    N.assert_rows_close(logits.grad, gref, N.CE_TOL, "dlogits")


@pytest.mark.parametrize("vocab", [1000, 1017, 1024 - 8])
def test_cross_entropy_padded_vocab(vocab):
    """Columns >= vocab are padding: excluded from the softmax and given zero gradient (same
    peaked inputs and row-relative criterion as test_cross_entropy)."""
    logits, tgt, dl = N.ce_case(200, 1024, vocab, device=DEV, seed=11)
    logits.requires_grad_()
    loss = SF.cross_entropy(logits, tgt, vocab_size=vocab)
    ref, gref = N.ce_ref(logits, tgt, dl, vocab)
    torch.testing.assert_close(loss, ref, atol=5e-3, rtol=1e-3)
    (loss * dl).sum().backward()
    N.assert_rows_close(logits.grad, gref, N.CE_TOL, "dlogits")
    assert logits.grad[:, vocab:].abs().max().item() == 0


@pytest.mark.parametrize("V,vocab", [(50304, 50257), (1000, 0), (33792, 0), (60000, 0)])
def test_lm_head_cross_entropy(V, vocab):
    """LM-head GEMM + ce_fused (row overwritten in place, dloss applied on the hidden side)
    against fp32 math on the same 16-bit logits, with peaked logits (std ~4), half the targets
    the argmax, an ignored row, vocab padding and O(1) signed dloss; dh and dW judged per row
    relative to the row max. Mutation check (tests/test_numerics_sensitivity.py): the softmax
    term dropped gives row-relative errors ~9-10, scaled x1.1 ~0.87-1.0, vs tol 0.03; a bf16
    emulation of this op's rounding points gives <= 0.009."""
    from smdt_amd.parallel import tensor_parallel as tp
    h, w, tgt, dl = N.lmce_case(96, 3, 256, V, vocab, device=DEV)
    h.requires_grad_()
    w.requires_grad_()
    assert tp.lm_head_ce_ok(h, w, 1)
    assert not tp.lm_head_ce_ok(h.detach().half(), w.detach().half(), 1)   # fp16: separate CE path
    lg16 = tp.linear_rows(h.detach(), w.detach())                # the GEMM the op runs, same kernel
    lgf = h.detach().float() @ w.detach().float().t()
    assert ((lg16.float() - lgf).abs() <= lgf.abs() * 2 ** -7 + 1e-3).all()
    loss = tp.LMHeadCrossEntropy.apply(h, w, tgt, -100, vocab if 0 < vocab < V else 0)
    ref, dhr, dwr = N.lmce_ref(h, w, lg16, tgt, dl, vocab)
    torch.testing.assert_close(loss, ref, atol=5e-3, rtol=1e-3)
    assert loss[3, 1].item() == 0
    (loss * dl).sum().backward()
    N.assert_rows_close(h.grad, dhr, N.CE_TOL, "dh")
    N.assert_rows_close(w.grad, dwr, N.CE_TOL, "dW")
    if vocab:
        assert w.grad[vocab:].abs().max().item() == 0


@pytest.mark.parametrize("V,vocab,ranks", [(50304, 50257, 2), (50432, 50257, 2), (4096, 0, 4)])
def test_vocab_parallel_lm_head_ce_two_shards(V, vocab, ranks):
    """VocabParallelLMHeadCE's math for ``ranks`` vocab shards in one process on the HIP kernel
    (ce_fused_kernel<LOCAL>: exp(x - m_local) in place + row statistics): combined loss, dh and dW
    against fp32 math on the same 16-bit logits, peaked logits, row-relative criterion (its
    mutation check: tests/test_numerics_sensitivity.py, vocab-parallel CPU twin included)."""
    from smdt_amd.parallel import tensor_parallel as tp
    h, w, tgt, dl = N.lmce_case(64, 3, 256, V, vocab, device=DEV)
    loss, dh, dw, lg = N.vp_lmce_two_shards(h, w, tgt, dl, vocab, ranks)
    rl, rdh, rdw = N.lmce_ref(h, w, lg, tgt, dl, vocab)
    torch.testing.assert_close(loss, rl, atol=5e-3, rtol=1e-3)
    N.assert_rows_close(dh, rdh, N.CE_TOL, "dh")
    N.assert_rows_close(dw, rdw, N.CE_TOL, "dW")
    # the kernel against its CPU reference on one shard (statistics and the in-place e)
    x = h.reshape(-1, h.shape[-1])
    lg0 = tp.linear_rows(x, w[: V // ranks])
    cpu = lg0.cpu().clone()
    st = tp.ce_local_pass(lg0, tgt.reshape(-1), 0, 0)
    stc = tp.ce_local_pass(cpu, tgt.reshape(-1).cpu(), 0, 0)
    torch.testing.assert_close(st.cpu(), stc, atol=1e-3, rtol=1e-3)
    torch.testing.assert_close(lg0.float().cpu(), cpu.float(), atol=1e-2, rtol=1e-2)


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("D", [64, 128])
@pytest.mark.parametrize("causal", [True, False])
@pytest.mark.parametrize("heads", [(4, 4), (8, 2)])
def test_flash_attention(D, causal, heads, dt):
    torch.manual_seed(10)
    B, S = 2, 256
    H, Hkv = heads
    q = torch.randn(B, S, H, D, device=DEV, dtype=dt, requires_grad=True)
    k = torch.randn(B, S, Hkv, D, device=DEV, dtype=dt, requires_grad=True)
    v = torch.randn(B, S, Hkv, D, device=DEV, dtype=dt, requires_grad=True)
    scale = 1 / math.sqrt(D)
    o = SF.flash_attention(q, k, v, scale, causal)
    qr, kr, vr = (t.detach().float().requires_grad_() for t in (q, k, v))
    orf = SF.attention_ref(qr, kr, vr, scale, causal)
    torch.testing.assert_close(o.float(), orf, atol=2e-2, rtol=2e-2)
    do = torch.randn_like(o)
    o.backward(do)
    orf.backward(do.float())
    for a, r in ((q, qr), (k, kr), (v, vr)):
        err = (a.grad.float() - r.grad).abs().max().item()
        assert err < 0.05 * max(1.0, r.grad.abs().max().item()), err


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("D", [64, 128])
@pytest.mark.parametrize("causal", [True, False])
@pytest.mark.parametrize("heads", [(4, 4), (8, 2)])
def test_flash_attention_dropout(D, causal, heads, dt):
    """In-kernel attention dropout == reference attention with the bit-exact twin of the
    kernels' keep-mask (forward and all three gradients)."""
    torch.manual_seed(12)
    B, S = 2, 256
    H, Hkv = heads
    p, seed, off = 0.1, 1234, 77
    q = torch.randn(B, S, H, D, device=DEV, dtype=dt, requires_grad=True)
    k = torch.randn(B, S, Hkv, D, device=DEV, dtype=dt, requires_grad=True)
    v = torch.randn(B, S, Hkv, D, device=DEV, dtype=dt, requires_grad=True)
    scale = 1 / math.sqrt(D)
    o = SF._FlashAttn.apply(q, k, v, scale, causal, p, seed, off)
    keep = SF.flash_dropout_keep_mask(B, H, S, p, seed, off, DEV)
    rate = 1 - keep.float().mean().item()
    assert abs(rate - SF.flash_dropout_thr(p)[0] / 128) < 0.01, rate
    qr, kr, vr = (t.detach().float().requires_grad_() for t in (q, k, v))
    orf = SF.attention_ref(qr, kr, vr, scale, causal, p, keep)
    torch.testing.assert_close(o.float(), orf, atol=2e-2, rtol=2e-2)
    do = torch.randn_like(o)
    o.backward(do)
    orf.backward(do.float())
    for a, r in ((q, qr), (k, kr), (v, vr)):
        err = (a.grad.float() - r.grad).abs().max().item()
        assert err < 0.05 * max(1.0, r.grad.abs().max().item()), err
    # a different offset gives a different mask; same (seed, offset) is reproducible
    o2 = SF._FlashAttn.apply(q.detach(), k.detach(), v.detach(), scale, causal, p, seed, off)
    o3 = SF._FlashAttn.apply(q.detach(), k.detach(), v.detach(), scale, causal, p, seed, off + 1)
    assert torch.equal(o2, o.detach()) and not torch.equal(o3, o2)


@pytest.mark.parametrize("S", [384, 512, 1024])
@pytest.mark.parametrize("causal", [True, False])
@pytest.mark.parametrize("p", [0.0, 0.1])
def test_flash_attention_d64_lengths(S, causal, p):
    """D = 64 at several lengths (one and several 128-row query blocks, every causal diagonal
    case, a length that is not a multiple of 256)."""
    torch.manual_seed(15)
    B, H, D = 2, 4, 64
    q, k, v = (torch.randn(B, S, H, D, device=DEV, dtype=torch.bfloat16, requires_grad=True) for _ in range(3))
    scale = 1 / math.sqrt(D)
    o = SF._FlashAttn.apply(q, k, v, scale, causal, p, 99, 5)
    keep = SF.flash_dropout_keep_mask(B, H, S, p, 99, 5, DEV) if p > 0 else None
    qr, kr, vr = (t.detach().float().requires_grad_() for t in (q, k, v))
    orf = SF.attention_ref(qr, kr, vr, scale, causal, p, keep) if p > 0 else SF.attention_ref(qr, kr, vr, scale, causal)
    torch.testing.assert_close(o.float(), orf, atol=2e-2, rtol=2e-2)
    do = torch.randn_like(o)
    o.backward(do)
    orf.backward(do.float())
    for a, r in ((q, qr), (k, kr), (v, vr)):
        err = (a.grad.float() - r.grad).abs().max().item()
        assert err < 0.05 * max(1.0, r.grad.abs().max().item()), err


def test_flash_attention_qkv_seq_first_matches_unfused():
    torch.manual_seed(11)
    S, B, nh, hd = 256, 2, 4, 64
    qkv = torch.randn(S, B, 3 * nh * hd, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    o = SF.flash_attention_qkv(qkv, nh, nh, hd, seq_first=True, causal=True)
    qr = qkv.detach().float().requires_grad_()
    q, k, v = SF._qkv_views(qr, nh, nh, hd, True)
    orf = SF.attention_ref(q, k, v, 1 / math.sqrt(hd), True).transpose(0, 1).flatten(-2)
    torch.testing.assert_close(o.float(), orf, atol=2e-2, rtol=2e-2)
    do = torch.randn_like(o)
    o.backward(do)
    orf.backward(do.float())
    err = (qkv.grad.float() - qr.grad).abs().max().item()
    assert err < 0.05 * max(1.0, qr.grad.abs().max().item())


def _attn_check(q, k, v, scale, causal, tol=0.05):
    o = SF.flash_attention(q, k, v, scale, causal)
    qr, kr, vr = (t.detach().float().requires_grad_() for t in (q, k, v))
    orf = SF.attention_ref(qr, kr, vr, scale, causal)
    err = (o.float() - orf).abs().max().item()
    assert err < 2e-2 * max(1.0, orf.abs().max().item()), err
    do = torch.randn_like(o)
    o.backward(do)
    orf.backward(do.float())
    for a, r in ((q, qr), (k, kr), (v, vr)):
        err = (a.grad.float() - r.grad).abs().max().item()
        assert err < tol * max(1.0, r.grad.abs().max().item()), err


@pytest.mark.parametrize("S,dt", [(1024, torch.bfloat16), (2048, torch.bfloat16), (2048, torch.float16)])
def test_flash_attention_production_shapes_gqa_d128(S, dt):
    """LLaMA / GPT-3 6.7B-like attention: D = 128, GQA 32 q / 8 kv heads, long sequences."""
    torch.manual_seed(13)
    B, H, Hkv, D = 1, 32, 8, 128
    q = torch.randn(B, S, H, D, device=DEV, dtype=dt, requires_grad=True)
    k = torch.randn(B, S, Hkv, D, device=DEV, dtype=dt, requires_grad=True)
    v = torch.randn(B, S, Hkv, D, device=DEV, dtype=dt, requires_grad=True)
    _attn_check(q, k, v, 1 / math.sqrt(D), True)


@pytest.mark.parametrize("S,D", [(200, 64), (256, 80), (130, 32)])
def test_flash_attention_padded_shapes_run_on_kernels(S, D):
    """Causal S % 128 != 0 and head dims outside {64, 128} are zero-padded onto the kernels (exact);
    nothing drops to the S x S reference on the GPU."""
    torch.manual_seed(14)
    B, H = 2, 4
    q, k, v = (torch.randn(B, S, H, D, device=DEV, dtype=torch.bfloat16, requires_grad=True) for _ in range(3))
    calls = []
    real = SF.attention_ref
    SF.attention_ref = lambda *a, **kw: calls.append(1) or real(*a, **kw)
    try:
        o = SF.flash_attention(q, k, v, 1 / math.sqrt(D), True)
    finally:
        SF.attention_ref = real
    assert not calls and o.shape == (B, S, H, D)
    _attn_check(q, k, v, 1 / math.sqrt(D), True)


def test_flash_attention_rejects_unsupported_on_gpu():
    q = torch.randn(1, 256, 4, 64, device=DEV, dtype=torch.float32)
    with pytest.raises(RuntimeError, match="bf16 / fp16"):
        SF.flash_attention(q, q, q, 0.125, True)
    qb = torch.randn(1, 200, 4, 64, device=DEV, dtype=torch.bfloat16)
    with pytest.raises(RuntimeError, match="multiple of 128"):
        SF.flash_attention(qb, qb, qb, 0.125, False)


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
def test_wgrad_mfma_fp16_and_bf16(dt):
    """Hand-written MFMA wgrad (single and grouped launch) in both 16-bit types vs fp32 matmul."""
    torch.manual_seed(15)
    C = _ext.ext()
    M, N, K = 2048, 1024, 768
    dy = torch.randn(M, N, device=DEV, dtype=dt)
    x = torch.randn(M, K, device=DEV, dtype=dt)
    ref = dy.float().t() @ x.float()
    mg = torch.ones(N, K, device=DEV, dtype=torch.float32)
    assert C.wgrad_mfma(mg, dy, x, 0)
    torch.testing.assert_close(mg, ref + 1, atol=0.05, rtol=1e-3)
    mg2 = torch.zeros(N, K, device=DEV, dtype=torch.float32)
    mg3 = torch.zeros(K, N, device=DEV, dtype=torch.float32)
    assert C.wgrad_grouped([mg2, mg3], [dy, x], [x, dy])
    torch.testing.assert_close(mg2, ref, atol=0.05, rtol=1e-3)
    torch.testing.assert_close(mg3, ref.t(), atol=0.05, rtol=1e-3)


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
def test_wgrad_grouped_bias_column_sums(dt):
    """The grouped wgrad launch also accumulates each problem's bias gradient (column sums of
    dY) into an fp32 target: whole tiles (plain read-modify-write), partial tiles (N = 1008, K = 520
    not multiples of 256), tail-split pieces (fp32 atomics), a problem without a bias in the same
    launch, and a second launch accumulating on top."""
    torch.manual_seed(16)
    C = _ext.ext()
    # 256 whole tiles of the first problem run the plain epilogue, the other 45 tiles the split tail
    shapes = [(2048, 4096, 4096), (4096, 1536, 1024), (2048, 1008, 520), (4096, 256, 256), (1024, 512, 1024)]
    dys = [torch.randn(M, N, device=DEV, dtype=dt) for M, N, _ in shapes]
    xs = [torch.randn(M, K, device=DEV, dtype=dt) for M, _, K in shapes]
    mgs = [torch.zeros(N, K, device=DEV) for _, N, K in shapes]
    bias = [torch.full((N,), 0.5, device=DEV) if i != 3 else torch.empty(0, device=DEV)
            for i, (_, N, _) in enumerate(shapes)]
    for rep in range(2):
        assert C.wgrad_grouped(mgs, dys, xs, bias)
    for i, (dy, x, mg) in enumerate(zip(dys, xs, mgs)):
        torch.testing.assert_close(mg, 2 * (dy.float().t() @ x.float()), atol=0.1, rtol=2e-3)
        if i != 3:
            torch.testing.assert_close(bias[i], 0.5 + 2 * dy.float().sum(0), atol=0.02, rtol=1e-4)


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("shape", [(1024, 1024), (3072, 1024), (1024, 4096), (50304, 1024), (200, 136), (8, 8)])
def test_transpose2d(dt, shape):
    x = torch.randn(*shape, device="cuda").to(dt)
    y = _ext.ext().transpose2d(x)
    assert y.shape == (shape[1], shape[0]) and y.is_contiguous()
    assert torch.equal(y, x.t().contiguous())


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
def test_linear_dgrad_tn_matches_nn(dt):
    """The TN dgrad (F.linear with a transposed weight copy) against fp32 dY @ W, through the
    Megatron linear autograd function."""
    from smdt_amd.parallel import tensor_parallel as tp
    torch.manual_seed(0)
    x = torch.randn(4, 256, 1024, device="cuda", dtype=dt, requires_grad=True)
    w = (torch.randn(3072, 1024, device="cuda") * 0.02).to(dt).requires_grad_(True)
    y = tp.LinearWithGradAccumulationAndAsyncCommunication.apply(x, w, None, False, False)
    g = torch.randn_like(y)
    y.backward(g)
    ref = g.float().matmul(w.float())
    err = (x.grad.float() - ref).abs().max().item()
    assert err <= 2e-2 * ref.abs().max().item(), err
    wt = tp._dgrad_weight_t(w.detach())
    assert wt is not None, "TN dgrad path not taken on the GPU"
    out = torch.empty_like(x.grad)
    tp.dgrad_into(out, g, w.detach(), wt)
    assert torch.equal(out, tp.dgrad(g, w.detach(), wt))



def test_dgrad_weight_t_cache_invalidation():
    """W^T is reused while the weight is unchanged, rebuilt after an in-place torch write (version
    counter) and after params_changed() (the optimizer's raw-kernel writes)."""
    from smdt_amd.parallel import tensor_parallel as tp
    w = torch.nn.Parameter(torch.randn(256, 128, device=DEV, dtype=torch.bfloat16))
    a = tp._dgrad_weight_t(w)
    assert a is tp._dgrad_weight_t(w)
    with torch.no_grad():
        w.add_(1.0)
    b = tp._dgrad_weight_t(w)
    assert b is not a and torch.equal(b, w.detach().t().contiguous())
    raw = w.detach().view(-1)
    _C().adam(torch.zeros(raw.numel(), device=DEV), torch.ones(raw.numel(), device=DEV),
              torch.zeros(raw.numel(), device=DEV), torch.zeros(raw.numel(), device=DEV), raw, 1e-3, 0.9, 0.95,
              1e-8, 0.0, 1, True, torch.ones(1, device=DEV), None)   # raw kernel write: no version bump
    tp.params_changed()
    c = tp._dgrad_weight_t(w)
    assert c is not b and torch.equal(c, w.detach().t().contiguous())


def test_graph_safe_dropout_rng():
    """With the device step counter registered (SF.enable_graph_rng) the flash and fused-LayerNorm
    dropout kernels mix its value into their keys at run time: the flash mask equals its bit-exact
    twin at that step (forward and all three gradients), a new step gives a new mask, and a
    captured HIP graph that advances the counter draws a fresh mask on every replay."""
    torch.manual_seed(21)
    B, S, H, D, p, seed, off = 2, 256, 4, 64, 0.1, 77, 5
    q, k, v = (torch.randn(B, S, H, D, device=DEV, dtype=torch.bfloat16, requires_grad=True) for _ in range(3))
    scale = 1 / math.sqrt(D)
    c = SF.enable_graph_rng()
    try:
        c.fill_(5)
        o = SF._FlashAttn.apply(q, k, v, scale, True, p, seed, off)
        keep = SF.flash_dropout_keep_mask(B, H, S, p, seed, off, DEV, step=5)
        assert not torch.equal(keep, SF.flash_dropout_keep_mask(B, H, S, p, seed, off, DEV))
        qr, kr, vr = (t.detach().float().requires_grad_() for t in (q, k, v))
        orf = SF.attention_ref(qr, kr, vr, scale, True, p, keep)
        torch.testing.assert_close(o.float(), orf, atol=2e-2, rtol=2e-2)
        do = torch.randn_like(o)
        o.backward(do)
        orf.backward(do.float())
        for a, r in ((q, qr), (k, kr), (v, vr)):
            err = (a.grad.float() - r.grad).abs().max().item()
            assert err < 0.05 * max(1.0, r.grad.abs().max().item()), err
        qd, kd, vd = q.detach(), k.detach(), v.detach()
        c.fill_(6)
        assert not torch.equal(SF._FlashAttn.apply(qd, kd, vd, scale, True, p, seed, off), o.detach())
        # captured: the replays see counter values 7, 8 (advanced inside the graph)
        c.fill_(6)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            SF.advance_graph_rng()
            og = SF._FlashAttn.apply(qd, kd, vd, scale, True, p, seed, off)
        outs = []
        for _ in range(2):
            g.replay()
            outs.append(og.clone())
        for st, got in zip((7, 8), outs):
            kp = SF.flash_dropout_keep_mask(B, H, S, p, seed, off, DEV, step=st)
            want = SF.attention_ref(qd.float(), kd.float(), vd.float(), scale, True, p, kp)
            torch.testing.assert_close(got.float(), want, atol=2e-2, rtol=2e-2)
        assert not torch.equal(outs[0], outs[1])
        # fused LayerNorm dropout: forward and backward agree at a step, differ across steps
        x = torch.randn(128, 1024, device=DEV, dtype=torch.bfloat16, requires_grad=True)
        res = torch.zeros(128, 1024, device=DEV, dtype=torch.bfloat16)
        gam = torch.ones(1024, device=DEV, dtype=torch.bfloat16, requires_grad=True)
        bet = torch.zeros(1024, device=DEV, dtype=torch.bfloat16, requires_grad=True)
        masks = []
        for st in (3, 4):
            c.fill_(st)
            # the same host (seed, offset) both times: only the device counter differs
            _, s_ = SF.bias_dropout_add_norm(x, None, res, gam, bet, 0.25, True, 1e-5, False, rng=SF.PhiloxState(9))
            x.grad = None
            s_.backward(torch.ones_like(s_))
            kept = s_ != 0
            assert torch.all(x.grad[~kept] == 0) and torch.all(x.grad[kept] != 0)
            masks.append(kept)
        assert not torch.equal(masks[0], masks[1])
    finally:
        SF.disable_graph_rng()


def test_paced_copy_copies_and_holds_for_its_link_time():
    """Link stand-in of the single-GPU rank emulation (csrc/kernels/link_standin.hip): an exact
    copy that does not finish before its modelled transfer time (and not grossly after it)."""
    from smdt_amd.ops import _ext
    C = _ext.ext()
    send = torch.randn(16 << 20, device="cuda", dtype=torch.bfloat16)      # 32 MB
    recv = torch.empty_like(send)
    C.paced_copy(recv, send, 64, 1000)
    torch.cuda.synchronize()
    assert torch.equal(recv, send)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for ns in (200_000, 1_000_000):
        s.record()
        C.paced_copy(recv, send, 64, ns)
        e.record()
        torch.cuda.synchronize()
        ms = s.elapsed_time(e)
        assert ns / 1e6 * 0.98 <= ms <= ns / 1e6 + 0.5, (ns, ms)
