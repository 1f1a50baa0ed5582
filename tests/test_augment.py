"""Oxford-Pet augmentations (data/augment.py) — statistical checks of each op on CPU, mirroring
the albumentations transforms of the reference pipeline (pytorch_oxford_ddp.py:140-160) — and the
recipe's util helpers (util.py: accuracy / meters / LR schedule)."""
import os
import sys
import types

import pytest
import torch

from smdt_amd.data import augment as A

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _img(n=4, h=64, w=64, seed=0):
    g = torch.Generator().manual_seed(seed)
    return torch.rand(n, 3, h, w, generator=g)


def _hf_energy(x):
    return (x[..., 1:, :] - x[..., :-1, :]).abs().mean() + (x[..., :, 1:] - x[..., :, :-1]).abs().mean()


def test_blurs_preserve_mean_and_remove_high_frequencies():
    x = _img()
    g = torch.Generator().manual_seed(1)
    for y in (A.box_blur(x), A.motion_blur(x, g), A.median_blur(x)):
        assert y.shape == x.shape
        assert abs(y.mean().item() - x.mean().item()) < 0.02
        assert _hf_energy(y) < 0.8 * _hf_energy(x)


def test_median_blur_removes_salt_noise():
    x = torch.full((1, 3, 32, 32), 0.5)
    x[0, :, 10, 10] = 1.0
    x[0, :, 20, 5] = 0.0
    y = A.median_blur(x)
    torch.testing.assert_close(y, torch.full_like(x, 0.5))


def test_motion_blur_kernel_is_a_normalised_line():
    x = torch.zeros(1, 3, 15, 15)
    x[0, :, 7, 7] = 1.0
    y = A.motion_blur(x, torch.Generator().manual_seed(3))
    assert abs(y.sum().item() - 3.0) < 1e-4                       # mass preserved per channel
    nz = (y[0, 0] > 1e-6).sum().item()
    assert 5 <= nz <= 21                                          # a thin line, not a box


def test_sharpen_and_emboss_raise_high_frequencies_within_range():
    x = A.box_blur(_img(seed=2))
    g = torch.Generator().manual_seed(4)
    for y in (A.sharpen(x, g), A.emboss(x, g)):
        assert y.min() >= 0 and y.max() <= 1
        assert _hf_energy(y) > 1.05 * _hf_energy(x)


def test_clahe_stretches_low_contrast_luma():
    g = torch.Generator().manual_seed(5)
    x = 0.45 + 0.1 * torch.rand(2, 3, 256, 256, generator=g)      # narrow luma range, 32x32 tiles
    y = A.clahe(x, clip_limit=2.0)
    luma = lambda t: 0.299 * t[:, 0] + 0.587 * t[:, 1] + 0.114 * t[:, 2]   # noqa: E731
    assert luma(y).std() > 2.0 * luma(x).std()
    assert y.min() >= 0 and y.max() <= 1
    # the clip limit bounds the stretch: clip 1 (no equalisation gain) changes little
    y1 = A.clahe(x, clip_limit=1.0)
    assert luma(y1).std() < luma(y).std()


def test_hsv_round_trip_and_hue_shift_keeps_value():
    x = _img(seed=6)
    torch.testing.assert_close(A.hsv_to_rgb(A.rgb_to_hsv(x)), x, atol=1e-5, rtol=1e-5)
    y = A.hue_saturation_value(x, torch.Generator().manual_seed(7), hue=20, sat=0, val=0)
    hx, hy = A.rgb_to_hsv(x), A.rgb_to_hsv(y)
    torch.testing.assert_close(hy[:, 2], hx[:, 2], atol=1e-5, rtol=1e-5)      # value untouched
    dh = ((hy[:, 0] - hx[:, 0] + 0.5) % 1.0 - 0.5)
    sat = hx[:, 1] > 0.2
    assert dh[sat].abs().max() <= 20 / 180 + 1e-4 and dh[sat].abs().mean() > 1e-3


def test_gauss_noise_std_matches_var_limit():
    x = torch.full((8, 3, 64, 64), 0.5)
    y = A.gauss_noise(x, torch.Generator().manual_seed(8), var_limit=(25.0, 25.0))
    assert abs((y - x).std().item() - 5.0 / 255) < 0.002


def test_one_of_applies_with_probability_and_weights():
    x = torch.zeros(4000, 1, 1, 1)
    g = torch.Generator().manual_seed(9)
    y = A.one_of(x, 0.5, [(3.0, lambda t: t + 1), (1.0, lambda t: t + 2)], g)
    frac = (y != 0).float().mean().item()
    assert abs(frac - 0.5) < 0.04
    ones, twos = (y == 1).sum().item(), (y == 2).sum().item()
    assert abs(ones / max(ones + twos, 1) - 0.75) < 0.05


def test_gpu_augment_train_pipeline_shapes_and_range():
    from smdt_amd.data.image_folder import GpuAugment
    aug = GpuAugment(out_size=(48, 48), train=True, noise_p=1.0, blur_p=1.0, color_p=1.0, hsv_p=1.0)
    x = (torch.rand(6, 3, 64, 80) * 255).to(torch.uint8)
    y = aug(x, torch.Generator().manual_seed(10))
    assert y.shape == (6, 3, 48, 48) and torch.isfinite(y).all()


def _util():
    sys.path.insert(0, os.path.join(ROOT, "recipes", "2_training_oxford-pet_ddp"))
    import util
    return util


def test_oxford_util_accuracy_meters_and_lr_schedule(capsys):
    util = _util()
    g = torch.Generator().manual_seed(11)
    out, tgt = torch.randn(64, 37, generator=g), torch.randint(0, 37, (64,), generator=g)
    top1, top5 = util.accuracy(out, tgt, (1, 5))
    ranks = (out > out.gather(1, tgt[:, None])).sum(1)        # rank of the true class
    assert top1.item() == pytest.approx(100 * (ranks < 1).float().mean().item())
    assert top5.item() == pytest.approx(100 * (ranks < 5).float().mean().item())
    m = util.AverageMeter("Loss", ":.3f")
    m.update(2.0, 3)
    m.update(1.0, 1)
    assert str(m) == "Loss 1.000 (1.750)"
    util.ProgressMeter(120, [m], prefix="Epoch: [1]").display(7)
    assert capsys.readouterr().out.strip() == "Epoch: [1][  7/120]\tLoss 1.000 (1.750)"
    opt = types.SimpleNamespace(param_groups=[{}, {}])
    args = types.SimpleNamespace(lr=0.1, rank=1)
    want = {(0, 0): 0.1 / 50, (4, 9): 0.1, (29, 0): 0.1, (30, 0): 0.01, (60, 0): 0.001, (80, 0): 1e-4, (90, 0): 1e-5}
    for (ep, st), lr in want.items():
        util.adjust_learning_rate(opt, ep, st, 10, args)
        assert opt.param_groups[1]["lr"] == pytest.approx(lr), (ep, st)
    assert util.to_python_float(torch.tensor([2.5])) == 2.5 and util.to_python_float([3]) == 3


@pytest.mark.gpu
def test_augment_prefetcher_matches_in_line_on_gpu():
    """AugmentPrefetcher (side stream + background thread) yields exactly the batches the in-line
    augmentation produces from the same generator state, and the step's stream sees them ready."""
    import itertools

    from smdt_amd.data.image_folder import AugmentPrefetcher, GpuAugment
    dev = torch.device("cuda")
    aug = GpuAugment((64, 64), train=True)
    src = torch.randint(0, 256, (8, 3, 80, 80), dtype=torch.uint8)
    tgt = torch.arange(8)
    g1 = torch.Generator(device=dev)
    g1.manual_seed(3)
    want = [aug(src.to(dev), g1) for _ in range(4)]
    g2 = torch.Generator(device=dev)
    g2.manual_seed(3)
    got = []
    for x, t in AugmentPrefetcher(itertools.islice(itertools.repeat((src, tgt)), 4), aug, dev, g2):
        got.append(x.clone())          # consumed on the current stream after the prefetcher's event
        assert torch.equal(t.cpu(), tgt)
    assert len(got) == 4
    for a, b in zip(got, want):
        assert torch.equal(a, b)


@pytest.mark.gpu
@pytest.mark.parametrize("ks", [3, 5, 7])
def test_aug_depthwise_kernel_matches_grouped_conv(ks):
    """csrc/kernels/augment.hip per-sample depthwise filter == the fp32 grouped-conv reference
    (reflect padding; odd image sizes cross tile edges)."""
    import torch.nn.functional as F
    from smdt_amd.ops import _ext
    g = torch.Generator(device="cuda").manual_seed(5)
    x = torch.rand(3, 3, 37, 61, device="cuda", generator=g)
    k = torch.randn(3, ks, ks, device="cuda", generator=g)
    y = _ext.ext().aug_depthwise(x, k)
    xp = F.pad(x.double(), (ks // 2,) * 4, mode="reflect")
    wgt = k.double()[:, None].expand(3, 3, ks, ks).reshape(9, 1, ks, ks)
    ref = F.conv2d(xp.reshape(1, 9, 37 + ks - 1, 61 + ks - 1), wgt, groups=9).view(3, 3, 37, 61)
    torch.testing.assert_close(y.double(), ref, rtol=1e-5, atol=1e-5)
    # the augment entry point takes the kernel on the GPU
    torch.testing.assert_close(A._depthwise(x, k).double(), ref, rtol=1e-5, atol=1e-5)


@pytest.mark.gpu
def test_aug_median3_kernel_matches_unfold_median():
    import torch.nn.functional as F
    from smdt_amd.ops import _ext
    g = torch.Generator(device="cuda").manual_seed(6)
    x = torch.rand(2, 3, 45, 33, device="cuda", generator=g)
    y = _ext.ext().aug_median3(x)
    p = F.unfold(F.pad(x, (1, 1, 1, 1), mode="reflect"), 3)
    ref = p.view(2, 3, 9, 45 * 33).median(dim=2).values.view(2, 3, 45, 33)
    assert torch.equal(y, ref)
    assert torch.equal(A.median_blur(x, 3), ref)
