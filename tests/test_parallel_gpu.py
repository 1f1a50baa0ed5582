"""GPU checks of the parallel-layer fast paths (single process, one MI355X)."""
import pytest
import torch

from smdt_amd.parallel import tensor_parallel as tp

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("fused", [True, False])
def test_wgrad_accumulates_into_fp32_main_grad(fused, monkeypatch):
    monkeypatch.setattr(tp, "_FUSED_WGRAD", fused)
    torch.manual_seed(0)
    out_f, in_f, tokens = 384, 256, 1000
    w = torch.nn.Parameter(torch.randn(out_f, in_f, device="cuda", dtype=torch.bfloat16))
    w.main_grad = torch.randn(out_f, in_f, device="cuda", dtype=torch.float32)
    base = w.main_grad.clone()
    ready = []
    w._smdt_grad_ready = lambda p: ready.append(p)
    g = torch.randn(tokens, out_f, device="cuda", dtype=torch.bfloat16)
    x = torch.randn(tokens, in_f, device="cuda", dtype=torch.bfloat16)
    r = tp._wgrad(w, g, x)
    assert r is None and len(ready) == 1
    ref = base + g.float().t() @ x.float()
    torch.testing.assert_close(w.main_grad, ref, atol=0.25, rtol=1e-2)


def test_linear_autograd_single_rank_matches_torch():
    torch.manual_seed(1)
    x = torch.randn(64, 8, 256, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    w = torch.nn.Parameter(torch.randn(512, 256, device="cuda", dtype=torch.bfloat16) * 0.02)
    b = torch.nn.Parameter(torch.zeros(512, device="cuda", dtype=torch.bfloat16))
    y = tp.linear_with_grad_accumulation_and_async_allreduce(x, w, b)
    xr = x.detach().float().requires_grad_()
    wr = w.detach().float().requires_grad_()
    yr = xr @ wr.t()
    torch.testing.assert_close(y.float(), yr, atol=5e-2, rtol=2e-2)
    dy = torch.randn_like(y)
    y.backward(dy)
    yr.backward(dy.float())
    torch.testing.assert_close(x.grad.float(), xr.grad, atol=5e-2, rtol=2e-2)
    torch.testing.assert_close(w.grad.float(), wr.grad, atol=0.5, rtol=2e-2)
