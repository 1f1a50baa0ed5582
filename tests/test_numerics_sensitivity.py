"""The kernel tests' criteria can fail (CPU twin of every mutation check).

For each numerics case used by ``test_kernels_gpu.py`` (cross entropy, padded-vocab CE, LM head +
CE, scaled / causal / masked softmax): an emulation of the kernel's rounding points passes the
row-relative criterion at the tolerance the GPU test uses, while a wrong implementation fails it:
softmax term dropped, softmax term x1.1, all-zero output, all-zero gradient, or a gradient that
is zero beyond row 64.
"""
import pytest
import torch

from _numerics import (CE_TOL, SOFTMAX_TOL, ce_case, ce_kernel_emulation, ce_ref, lmce_case,
                       lmce_kernel_emulation, lmce_ref, row_rel_err, softmax_case, softmax_grad_floor,
                       softmax_ref)


@pytest.mark.parametrize("V,vocab", [(50304, 0), (1000, 0), (1024, 1017)])
def test_ce_criterion_rejects_mutations(V, vocab):
    logits, tgt, dl = ce_case(300 if V > 2000 else 200, V, vocab)
    _, good = ce_ref(logits, tgt, dl, vocab)
    _, emu = ce_kernel_emulation(logits, tgt, dl, vocab)
    assert row_rel_err(emu, good) <= CE_TOL / 3
    for soft in (0.0, 1.1, 0.9):
        _, bad = ce_ref(logits, tgt, dl, vocab, soft=soft)
        assert row_rel_err(bad, good) > 2 * CE_TOL, soft


@pytest.mark.parametrize("V,vocab", [(50304, 50257), (1000, 0)])
def test_lm_head_ce_criterion_rejects_mutations(V, vocab):
    h, w, tgt, dl = lmce_case(s=48, b=3, V=V, vocab=vocab)
    lg = (h.float().reshape(-1, h.shape[-1]) @ w.float().t()).bfloat16()
    loss, dh, dw = lmce_ref(h, w, lg, tgt, dl, vocab)
    eloss, edh, edw = lmce_kernel_emulation(h, w, lg, tgt, dl, vocab)
    assert (eloss - loss).abs().max().item() < 1e-3
    assert row_rel_err(edh, dh) <= CE_TOL / 3, row_rel_err(edh, dh)
    assert row_rel_err(edw, dw) <= CE_TOL / 3, row_rel_err(edw, dw)
    for soft in (0.0, 1.1):
        _, bdh, bdw = lmce_ref(h, w, lg, tgt, dl, vocab, soft=soft)
        assert row_rel_err(bdh, dh) > 2 * CE_TOL, (soft, row_rel_err(bdh, dh))
        assert row_rel_err(bdw, dw) > 2 * CE_TOL, (soft, row_rel_err(bdw, dw))


@pytest.mark.parametrize("sk", [128, 1024])
@pytest.mark.parametrize("causal", [True, False])
def test_softmax_criterion_rejects_mutations(sk, causal):
    x, dy = softmax_case(sk, causal, b=1, np_=2)
    y, dx = softmax_ref(x, dy, 0.125, causal)
    # kernel emulation: y stored 16-bit, dx = scale * y (dy - sum(dy y)) from the 16-bit y, stored 16-bit
    yb = y.bfloat16().float()
    dxe = (0.125 * yb * (dy.float() - (dy.float() * yb).sum(-1, keepdim=True))).bfloat16()
    assert row_rel_err(yb, y) <= SOFTMAX_TOL / 3
    fl = softmax_grad_floor(y, dy, 0.125)
    assert row_rel_err(dxe, dx, row_floor=fl) <= SOFTMAX_TOL / 3, row_rel_err(dxe, dx, row_floor=fl)
    assert row_rel_err(torch.zeros_like(y), y) > 2 * SOFTMAX_TOL
    assert row_rel_err(torch.zeros_like(dx), dx, row_floor=fl) > 2 * SOFTMAX_TOL
    assert row_rel_err(1.1 * dx, dx, row_floor=fl) > 2 * SOFTMAX_TOL
    cut = dx.clone()
    cut[..., 64:, :] = 0
    assert row_rel_err(cut, dx, row_floor=fl) > 2 * SOFTMAX_TOL


def test_masked_softmax_criterion_rejects_mutations():
    g = torch.Generator().manual_seed(6)
    x = (8 * torch.randn(2, 3, 64, 256, generator=g)).bfloat16()
    mask = torch.rand(2, 1, 64, 256, generator=g) < 0.3
    dy = torch.randn(2, 3, 64, 256, generator=g).bfloat16()
    y, dx = softmax_ref(x, dy, 0.125, False, mask)
    assert row_rel_err(y.bfloat16(), y) <= SOFTMAX_TOL / 3
    unmasked = torch.softmax(x.float() * 0.125, -1)
    assert row_rel_err(unmasked, y) > 2 * SOFTMAX_TOL
    assert row_rel_err(1.1 * dx, dx, row_floor=softmax_grad_floor(y, dy, 0.125)) > 2 * SOFTMAX_TOL


@pytest.mark.parametrize("V,vocab", [(50304, 50257), (1024, 0)])
def test_vocab_parallel_lm_head_ce_math_cpu(V, vocab):
    """CPU twin of test_kernels_gpu.test_vocab_parallel_lm_head_ce_two_shards: the two-shard math
    (local pass, combined statistics, one-hot at one element, hidden-side scale) equals the fp32
    reference on the same 16-bit logits within the criterion, and the same math with the
    softmax term mutated would not."""
    h, w, tgt, dl = lmce_case(s=32, b=3, V=V, vocab=vocab)
    from _numerics import vp_lmce_two_shards
    loss, dh, dw, lg = vp_lmce_two_shards(h, w, tgt, dl, vocab)
    rl, rdh, rdw = lmce_ref(h, w, lg, tgt, dl, vocab)
    assert (loss - rl).abs().max().item() < 1e-3
    assert row_rel_err(dh, rdh) <= CE_TOL / 3, row_rel_err(dh, rdh)
    assert row_rel_err(dw, rdw) <= CE_TOL / 3, row_rel_err(dw, rdw)
    _, bdh, bdw = lmce_ref(h, w, lg, tgt, dl, vocab, soft=1.1)
    assert row_rel_err(bdh, rdh) > 2 * CE_TOL and row_rel_err(bdw, rdw) > 2 * CE_TOL
