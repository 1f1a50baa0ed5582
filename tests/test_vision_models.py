"""Vision model zoo (ResNet family, Swin) — torchvision-compatible names and sizes (the reference
builds them with ``torchvision.models.__dict__[name]``, pytorch_oxford_ddp.py / util.py:241-246)."""
import pytest
import torch

from smdt_amd.models import zoo


@pytest.mark.parametrize("name,params", [("resnet50", 25_557_032), ("resnet18", 11_689_512),
                                         ("swin_b", 87_768_224), ("swin_t", 28_288_354)])
def test_param_counts_match_torchvision(name, params):
    m = zoo.create(name, 1000)
    assert sum(p.numel() for p in m.parameters()) == params


def test_swin_state_dict_uses_torchvision_names():
    keys = set(zoo.create("swin_t", 10).state_dict())
    for k in ("features.0.0.weight", "features.0.2.weight", "features.1.0.attn.relative_position_bias_table",
              "features.1.1.attn.qkv.weight", "features.2.reduction.weight", "features.2.norm.weight",
              "features.7.1.mlp.3.weight", "norm.weight", "head.weight"):
        assert k in keys, k


def test_swin_forward_backward_and_eval_determinism():
    torch.manual_seed(0)
    m = zoo.create("swin_t", 37)
    x = torch.randn(2, 3, 128, 128)
    y = m(x)
    assert y.shape == (2, 37)
    y.sum().backward()
    assert m.features[1][0].attn.relative_position_bias_table.grad is not None
    m.eval()
    with torch.no_grad():
        torch.testing.assert_close(m(x), m(x))


def test_shifted_window_mask_blocks_cross_region_attention():
    from smdt_amd.models.swin import ShiftedWindowAttention
    a = ShiftedWindowAttention(32, 7, 3, 2)
    b = a._bias(14, 14, 3, torch.device("cpu"), torch.float32)
    assert b.shape == (4, 2, 49, 49)
    # the last window (bottom-right) mixes 4 regions after the roll: some pairs are masked
    assert (b[3] < -50).any() and not (b[0] < -50).any()


def test_ddp_keeps_channels_last_weights():
    """DDP's flat param / grad buffers keep a channels-last conv weight's strides (the Oxford recipe
    moves the model to channels-last before wrapping it), and grads match an unwrapped copy."""
    import torch
    from smdt_amd.parallel.distributed import DistributedDataParallel as DDP

    torch.manual_seed(0)

    def net():
        return torch.nn.Sequential(torch.nn.Conv2d(3, 8, 3), torch.nn.ReLU(), torch.nn.Flatten(),
                                   torch.nn.Linear(8 * 6 * 6, 4))

    m = net()
    m2 = net()
    m2.load_state_dict(m.state_dict())
    m = m.to(memory_format=torch.channels_last)
    d = DDP(m, torch_compat=True)
    assert m[0].weight.is_contiguous(memory_format=torch.channels_last)
    for a, b in zip(m.parameters(), m2.parameters()):
        assert torch.equal(a, b)
    x = torch.randn(2, 3, 8, 8).to(memory_format=torch.channels_last)
    d(x).sum().backward()
    m2(x.contiguous()).sum().backward()
    for a, b in zip(m.parameters(), m2.parameters()):
        torch.testing.assert_close(a.grad, b.grad)
