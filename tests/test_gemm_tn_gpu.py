"""The hand-written TN GEMM (csrc/kernels/gemm_tn.hip) against a plain fp32 PyTorch reference:
out = a . b^T with the none / bias / bias + GeLU-tanh epilogues. Shapes cover one tile, a
partial last round of tiles, several tiles per persistent workgroup (max_blocks forces the
tile loop, the DMA stream across tile boundaries and the trickled epilogue), and K = 128 (four
32-deep stages per tile, the shortest stream). Asymmetric operands (an identity-like a with a non-symmetric b would hide a
transposed store; random data does not).
"""
import pytest
import torch

from smdt_amd.ops import _ext

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _ref_gelu(z):
    return torch.nn.functional.gelu(z, approximate="tanh")


def _rel(got, ref):
    return ((got.float() - ref).abs().max() / ref.abs().max().clamp_min(1e-6)).item()


@pytest.mark.parametrize("M,N,K,blocks", [
    (256, 256, 128, 0),          # one tile, 4 stages (the shortest supported K)
    (512, 768, 384, 0),          # 6 tiles, stages not a power of two
    (1024, 1024, 256, 3),        # 16 tiles over 3 persistent workgroups (5-6 tiles each)
    (2048, 512, 1024, 5),        # 16 tiles over 5 workgroups, 32 stages per tile
    (1024, 1024, 384, 3),        # the shortest trickled tile (12 stages) over several tiles
    (4096, 4096, 128, 0),        # 256 tiles: one full round of the chip
    (8192, 1280, 512, 0),        # 160 tiles
])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_gemm_tn_plain(M, N, K, blocks, dtype):
    C = _ext.ext()
    g = torch.Generator(device=DEV).manual_seed(M + N + K)
    a = torch.randn(M, K, device=DEV, dtype=dtype, generator=g)
    b = torch.randn(N, K, device=DEV, dtype=dtype, generator=g) * 0.1
    assert C.gemm_tn_supported(a, b)
    out = C.gemm_tn(a, b, 0, None, None, None, blocks)[0]
    ref = a.float() @ b.float().t()
    assert _rel(out, ref) < 1e-2
    # every element, not only the max: a wrong tile shows up as a large error count
    bad = ((out.float() - ref).abs() > 0.02 * ref.abs().max()).sum().item()
    assert bad == 0


@pytest.mark.parametrize("K,blocks", [(512, 0), (512, 7), (256, 5)])
def test_gemm_tn_bias_and_bias_gelu(K, blocks):
    """K >= 384: the tile's last 4 row blocks are stored during the next tile (trickled); K = 256:
    every block at the tile's end. The activation is computed from the rounded pre-activation, as
    the unfused bias_act_fwd pass does, so it must match that pass to rounding."""
    C = _ext.ext()
    torch.manual_seed(1)
    M, N = 2048, 1536
    a = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
    b = torch.randn(N, K, device=DEV, dtype=torch.bfloat16) * 0.05
    bias = torch.randn(N, device=DEV, dtype=torch.bfloat16)
    acc = a.float() @ b.float().t()
    ob = C.gemm_tn(a, b, 1, bias, None, None, blocks)[0]
    assert _rel(ob, acc + bias.float()) < 1e-2
    pre, act = C.gemm_tn(a, b, 2, bias, None, None, blocks)
    assert _rel(pre, acc) < 1e-2
    ref_act = _ref_gelu(acc + bias.float())
    assert (act.float() - ref_act).abs().max().item() < 3e-2 * ref_act.abs().max().item()
    unf = C.bias_act_fwd(pre, bias, 0)
    assert (act.float() - unf.float()).abs().max().item() <= 1e-2 * ref_act.abs().max().item()


def test_gemm_tn_into_given_buffers_and_unsupported():
    C = _ext.ext()
    torch.manual_seed(2)
    a = torch.randn(512, 256, device=DEV, dtype=torch.bfloat16)
    b = torch.randn(512, 256, device=DEV, dtype=torch.bfloat16)
    big = torch.zeros(2, 512, 512, device=DEV, dtype=torch.bfloat16)
    C.gemm_tn(a, b, 0, None, big[1], None, 0)
    assert big[0].abs().max().item() == 0
    assert _rel(big[1], a.float() @ b.float().t()) < 1e-2
    # shapes off the 256 / 128 grid are refused (the caller takes the library GEMM)
    assert not C.gemm_tn_supported(torch.randn(300, 256, device=DEV, dtype=torch.bfloat16), b)
    assert not C.gemm_tn_supported(a[:, :192].contiguous(), b[:, :192].contiguous())
    assert not C.gemm_tn_supported(a.float(), b.float())


@pytest.mark.parametrize("blocks", [0, 3])
def test_gemm_tn_gelu_backward_epilogue(blocks):
    """EPI_DGELU: out = (a . b^T) * gelu_tanh'(pre + bias), against the unfused path (the product
    rounded to 16 bits, then bias_act_bwd) and the fp32 reference."""
    C = _ext.ext()
    torch.manual_seed(3)
    M, N, K = 2048, 1024, 512
    a = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
    b = torch.randn(N, K, device=DEV, dtype=torch.bfloat16) * 0.05
    bias = torch.randn(N, device=DEV, dtype=torch.bfloat16)
    pre = torch.randn(M, N, device=DEV, dtype=torch.bfloat16) * 2
    got = C.gemm_tn(a, b, 3, bias, None, None, blocks, 0, pre)[0]
    prod = a.float() @ b.float().t()
    z = (pre.float() + bias.float()).requires_grad_()
    torch.nn.functional.gelu(z, approximate="tanh").backward(torch.ones_like(z))
    ref = prod * z.grad
    assert _rel(got, ref) < 2e-2
    unf = C.bias_act_bwd(prod.to(torch.bfloat16), pre, bias, 0, False, None)[0]
    assert (got.float() - unf.float()).abs().max().item() <= 1e-2 * ref.abs().max().item()


@pytest.mark.parametrize("mode", ["fused_mlp", "fused_fc1", "all_linears"])
def test_gpt_step_on_gemm_tn_matches_fp32_reference(monkeypatch, mode):
    """The flagship GPT step with both GeLU halves in the GEMMs ("fused_mlp": FusedGeLUMLP), with
    only fc1 + bias + GeLU fused ("fused_fc1"), and with every supported forward / dgrad linear on
    gemm_tn as well ("all_linears"), against the fp32 PyTorch reference (the peaked-head case of
    test_model_gpu, whose gradients check every parameter). The fused paths must actually run:
    their calls are counted."""
    import test_model_gpu as T
    from smdt_amd.parallel import tensor_parallel as tp
    monkeypatch.setattr(tp, "_FUSED_BIAS_GELU", True)
    monkeypatch.setattr(tp, "_fills_chip", lambda rows, n: True)   # test shapes: a few tiles only
    if mode == "all_linears":
        monkeypatch.setattr(tp, "_GEMM_TN", "1")
        monkeypatch.setattr(tp, "_GEMM_TN_SHAPES", None)
    calls = {"fc1": 0, "mlp": 0}
    orig_fc1, orig_mlp = tp.linear_bias_gelu, tp.FusedGeLUMLP.forward

    def counted_fc1(x, layer):
        calls["fc1"] += 1
        return orig_fc1(x, layer)

    def counted_mlp(ctx, *args):
        calls["mlp"] += 1
        return orig_mlp(ctx, *args)
    monkeypatch.setattr(tp, "linear_bias_gelu", counted_fc1)
    monkeypatch.setattr(tp.FusedGeLUMLP, "forward", staticmethod(counted_mlp))
    if mode == "fused_fc1":
        monkeypatch.setattr(tp, "fused_gelu_mlp_ok", lambda x, mlp: False)
    T.test_gpt_step_matches_fp32_reference(torch.bfloat16, True)
    if mode == "fused_fc1":
        assert calls == {"fc1": 2, "mlp": 0}   # both layers' MLPs
    else:
        assert calls == {"fc1": 0, "mlp": 2}


def _emulated_tp2_sp_gpt_grads(fused, monkeypatch):
    """One process as TP rank 0 of a tp2 + SP GPT (loopback TP group, ring collective-matmul
    linears): one forward + backward with dropout off; the loss and the fp32 main_grad buffer.
    SP chunks of 128 x 4 = 512 rows and a local 4h of 512: every chunk GEMM is a gemm_tn shape."""
    from smdt_amd.models.gpt import GPTModel
    from smdt_amd.models.transformer import TransformerConfig
    from smdt_amd.parallel import state as ps
    from smdt_amd.parallel import tensor_parallel as tp
    from smdt_amd.parallel.distributed import DistributedDataParallel as DDP
    monkeypatch.setattr(tp, "_FUSED_BIAS_GELU", fused)
    monkeypatch.setattr(tp, "_fills_chip", lambda rows, n: True)   # test shapes: a few tiles only
    calls = {"n": 0}
    orig = tp.SPFusedGeLUMLP.forward

    def counted(ctx, *args):
        calls["n"] += 1
        return orig(ctx, *args)
    monkeypatch.setattr(tp.SPFusedGeLUMLP, "forward", staticmethod(counted))
    ps.destroy_model_parallel()
    ps.initialize_emulated_tensor_parallel(2, 1)
    try:
        cfg = TransformerConfig(num_layers=2, hidden_size=256, num_attention_heads=4, padded_vocab_size=1024,
                                max_position_embeddings=256, hidden_dropout=0.0, attention_dropout=0.0,
                                params_dtype=torch.bfloat16, sequence_parallel=True, seed=7)
        model = GPTModel(cfg, device="cuda")
        ddp = DDP(model, grad_dtype=torch.float32)
        g = torch.Generator(device="cuda").manual_seed(13)
        t = torch.randint(0, 1000, (4, 257), device="cuda", generator=g)
        ddp.zero_grad_buffer()
        loss = model(t[:, :-1], labels=t[:, 1:]).float().mean()
        loss.backward()
        ddp.finish_grad_sync()
        torch.cuda.synchronize()
        return loss.item(), ddp.grad_data.clone(), calls["n"]
    finally:
        ps.destroy_model_parallel()


def test_sp_fused_gelu_mlp_matches_unfused(monkeypatch):
    """SPFusedGeLUMLP (TP > 1 + SP: fc1 bias-GeLU and fc2-dgrad GeLU-backward epilogues in the
    ring-chunk GEMMs) against the unfused column / row SP linears + bias_act passes on the same
    emulated tp2 rank: loss and every parameter's fp32 gradient (fc1 weight and bias, fc2 weight,
    and everything upstream of the MLP through d(x)). The fused path must run (counted) and the
    unfused one must not take it. Mutation check: dropping the GeLU derivative from the EPI_DGELU
    epilogue (d(pre) = dY W2) moves the fc1 gradients by O(1) of their max and fails here."""
    lf, gf, nf = _emulated_tp2_sp_gpt_grads(True, monkeypatch)
    lu, gu, nu = _emulated_tp2_sp_gpt_grads(False, monkeypatch)
    assert nf == 2 and nu == 0
    assert abs(lf - lu) <= 2e-3 * abs(lu)
    scale = gu.abs().max().item()
    assert scale > 0
    assert (gf - gu).abs().max().item() <= 2e-2 * scale
    # every parameter, relative to its own magnitude
    assert torch.linalg.vector_norm(gf - gu).item() <= 2e-2 * torch.linalg.vector_norm(gu).item()


def test_sp_ring_pieces_match_whole_chunks(monkeypatch):
    """The emulated tp2 + SP rank with every ring exchange in 2 row pieces (SMDT_RING_PIECES=2:
    the fused MLP's gemm_tn chunk GEMMs and the other ring GEMMs run per piece, at row offsets)
    gives the whole-chunk run's loss and fp32 gradients."""
    from smdt_amd.parallel import tensor_parallel as tp
    lw, gw, _ = _emulated_tp2_sp_gpt_grads(True, monkeypatch)
    monkeypatch.setattr(tp, "_RING_PIECES", 2)
    tp.SPLIT_STATS.pop("ring_pieces", None)
    lp, gp, _ = _emulated_tp2_sp_gpt_grads(True, monkeypatch)
    assert tp.SPLIT_STATS.get("ring_pieces", 0) > 0
    assert abs(lp - lw) <= 1e-3 * abs(lw)
    scale = gw.abs().max().item()
    assert (gp - gw).abs().max().item() <= 1e-2 * scale
