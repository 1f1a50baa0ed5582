"""End-to-end GPU numerics of the flagship GPT path: a full forward + backward through the gfx950
kernels (fused LN, flash attention, bias-GeLU, vocab CE, MFMA wgrad into fp32 main_grad) against
the same weights run in fp32 by the PyTorch reference path, in bf16 and fp16; and the reference's
Megatron recipe flags (NB3, ``--fp16``) running pretrain_gpt.py on the kernels."""
import os
import subprocess
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("dt,peaked", [(torch.bfloat16, False), (torch.float16, False), (torch.bfloat16, True)])
def test_gpt_step_matches_fp32_reference(dt, peaked):
    """``peaked``: the tied word embeddings are scaled x3, so the LM-head softmax puts ~0.8 on one
    column (mean row max) and the softmax term is ~64 % of the dlogits norm (at init it is ~3 %,
    below this test's 3e-2 threshold): a wrong softmax half of the fused LM-head CE backward then
    shows in every parameter's gradient."""
    from smdt_amd.models.gpt import GPTModel
    from smdt_amd.models.transformer import TransformerConfig
    from smdt_amd.parallel import state as ps
    from smdt_amd.parallel.distributed import DistributedDataParallel
    ps.destroy_model_parallel()
    kw = dict(num_layers=2, hidden_size=256, num_attention_heads=4, max_position_embeddings=256,
              padded_vocab_size=1024, hidden_dropout=0.0, attention_dropout=0.0, seed=3)
    ref = GPTModel(TransformerConfig(**kw, params_dtype=torch.float32))            # CPU, fp32
    gpu = GPTModel(TransformerConfig(**kw, params_dtype=dt), device="cuda")
    with torch.no_grad():
        for (n, pr), (_, pg) in zip(ref.named_parameters(), gpu.named_parameters()):
            pg.copy_(pr.to(dt))                                                      # same weights
        if peaked:
            gpu.embedding.weight.mul_(3)
        for pr, pg in zip(ref.parameters(), gpu.parameters()):
            pr.copy_(pg.float().cpu())                                               # rounded alike
    ddp = DistributedDataParallel(gpu)
    g = torch.Generator().manual_seed(4)
    toks = torch.randint(0, 1000, (4, 257), generator=g)
    loss_ref = ref(toks[:, :-1], labels=toks[:, 1:])
    loss_ref.mean().backward()
    ddp.zero_grad_buffer()
    loss = gpu(toks[:, :-1].cuda(), labels=toks[:, 1:].cuda())
    loss.float().mean().backward()
    ddp.finish_grad_sync()
    torch.testing.assert_close(loss.float().cpu(), loss_ref.detach(), atol=0.1 if peaked else 3e-2, rtol=1e-2)
    if peaked:                                  # the softmax term is a visible part of dlogits
        lg = ref.lm_logits(ref.decoder(ref._embed(toks[:, :-1], None, 0), None, None)).detach()
        assert torch.softmax(lg.float(), -1).amax(-1).mean() > 0.5
    for (n, pr), pg in zip(ref.named_parameters(), gpu.parameters()):
        got = pg.main_grad.float().cpu()
        want = pr.grad
        err = (got - want).norm() / want.norm().clamp_min(1e-12)
        assert err < 3e-2, (n, err.item())


def test_pretrain_gpt_nb3_fp16_flags_on_kernels(tmp_path):
    """NB3's Megatron flags (--fp16, fused kernels, flash attention) for 3 iterations: attention
    must run on the fp16 flash kernels (a GPU tensor never falls back to the S x S reference)."""
    script = os.path.join(ROOT, "recipes", "3_training_megatron-lm", "pretrain_gpt.py")
    args = ["--num-layers", "2", "--hidden-size", "256", "--num-attention-heads", "4", "--seq-length", "512",
            "--max-position-embeddings", "512", "--micro-batch-size", "4", "--global-batch-size", "8",
            "--lr", "0.0005", "--lr-decay-style", "cosine", "--lr-warmup-iters", "1", "--weight-decay", "0.1",
            "--adam-beta2", "0.999", "--fp16", "true", "--mock-data", "--log-interval", "1", "--eval-interval", "100",
            "--eval-iters", "1", "--train-iters", "3", "--vocab-size", "1024", "--tokenizer-type", "NullTokenizer",
            "--use-flash-attn"]
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT="29537",
               SMDT_ASSERT_FLASH="1")
    r = subprocess.run([sys.executable, script] + args, env=env, capture_output=True, text=True, timeout=300,
                       cwd=str(tmp_path))
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    out = " ".join(r.stdout.split())
    assert "iteration 3/ 3" in out or "iteration 3/3" in out, out[-2000:]
    import math
    import re
    last = out.split("iteration 3/")[-1]
    loss = float(re.search(r"lm loss: ([0-9.eE+-]+|NAN|nan)", last).group(1))
    assert math.isfinite(loss), last[:400]




@pytest.mark.parametrize("one_p,post_ln", [(True, False), (False, True)])
def test_gpt_model_form_variants_match_fp32_reference(one_p, post_ln):
    """``--apply-layernorm-1p`` (the fused norm kernel reads 1 + stored gamma) and
    ``--apply-residual-connection-post-layernorm`` (residual = norm output) through the bf16
    kernels: loss and every gradient against the same weights on the fp32 PyTorch path."""
    from smdt_amd.models.gpt import GPTModel
    from smdt_amd.models.transformer import TransformerConfig
    from smdt_amd.parallel import state as ps
    from smdt_amd.parallel.distributed import DistributedDataParallel
    ps.destroy_model_parallel()
    kw = dict(num_layers=2, hidden_size=256, num_attention_heads=4, max_position_embeddings=256,
              padded_vocab_size=1024, hidden_dropout=0.0, attention_dropout=0.0, seed=3,
              layernorm_zero_centered_gamma=one_p, apply_residual_connection_post_layernorm=post_ln)
    ref = GPTModel(TransformerConfig(**kw, params_dtype=torch.float32))
    gpu = GPTModel(TransformerConfig(**kw, params_dtype=torch.bfloat16), device="cuda")
    g = torch.Generator().manual_seed(5)
    with torch.no_grad():
        for n, pr in ref.named_parameters():
            if "norm.weight" in n:                     # gamma away from its init value
                pr.add_(0.2 * torch.randn(pr.shape, generator=g))
        for pr, pg in zip(ref.parameters(), gpu.parameters()):
            pg.copy_(pr.to(torch.bfloat16))
            pr.copy_(pg.float().cpu())
    ddp = DistributedDataParallel(gpu)
    toks = torch.randint(0, 1000, (4, 257), generator=g)
    loss_ref = ref(toks[:, :-1], labels=toks[:, 1:])
    loss_ref.mean().backward()
    ddp.zero_grad_buffer()
    loss = gpu(toks[:, :-1].cuda(), labels=toks[:, 1:].cuda())
    loss.float().mean().backward()
    ddp.finish_grad_sync()
    torch.testing.assert_close(loss.float().cpu(), loss_ref.detach(), atol=3e-2, rtol=1e-2)
    for (n, pr), pg in zip(ref.named_parameters(), gpu.parameters()):
        err = (pg.main_grad.float().cpu() - pr.grad).norm() / pr.grad.norm().clamp_min(1e-12)
        assert err < 3e-2, (n, err.item())


def test_switch_mlp_on_kernels_matches_per_expert_composition():
    """``--num-experts`` on the GPU: the sorted-slice Switch MLP (bf16 expert MLPs on the fused
    kernels) equals each token's expert run by itself on the same device, and backward runs."""
    from smdt_amd.models.transformer import SwitchMLP, TransformerConfig
    from smdt_amd.parallel import state as ps
    ps.destroy_model_parallel()
    cfg = TransformerConfig(num_layers=2, hidden_size=256, num_attention_heads=4, max_position_embeddings=256,
                            padded_vocab_size=1024, hidden_dropout=0.0, attention_dropout=0.0, seed=3,
                            num_experts=4, params_dtype=torch.bfloat16)
    mlp = SwitchMLP(cfg, 1, device="cuda")
    with torch.no_grad():
        mlp.router.mul_(20)
    x = torch.randn(128, 4, 256, device="cuda", generator=torch.Generator(device="cuda").manual_seed(0))
    x = x.to(torch.bfloat16).requires_grad_(True)
    out, _ = mlp(x)
    flat = x.detach().reshape(-1, 256)
    p, e = mlp.route(flat)
    assert len(set(e.tolist())) == 4
    want = torch.empty_like(flat)
    with torch.no_grad():
        for i in range(4):
            idx = (e == i).nonzero().view(-1)
            y, yb = mlp.experts[i](flat[idx].unsqueeze(1))
            want[idx] = ((y.squeeze(1) + yb) * p[idx].unsqueeze(-1).to(y.dtype))
    torch.testing.assert_close(out.reshape(-1, 256).float(), want.float(), atol=2e-2, rtol=2e-2)
    out.float().square().sum().backward()
    assert torch.isfinite(x.grad.float()).all() and mlp.router.grad.abs().sum() > 0


def test_use_cpu_initialization_gives_the_cpu_weights_on_the_gpu():
    """``--use-cpu-initialization``: the weights are drawn by the host generator and moved, so a
    GPU model starts from exactly the CPU model's weights (the device generator's draws differ)."""
    from smdt_amd.models.gpt import GPTModel
    from smdt_amd.models.transformer import TransformerConfig
    from smdt_amd.parallel import state as ps
    ps.destroy_model_parallel()
    kw = dict(num_layers=2, hidden_size=256, num_attention_heads=4, max_position_embeddings=256,
              padded_vocab_size=1024, seed=3, params_dtype=torch.bfloat16)
    cpu = GPTModel(TransformerConfig(**kw))
    gpu = GPTModel(TransformerConfig(**kw, use_cpu_initialization=True), device="cuda")
    dev = GPTModel(TransformerConfig(**kw), device="cuda")
    for (n, pc), pg, pd in zip(cpu.named_parameters(), gpu.parameters(), dev.parameters()):
        assert pg.is_cuda and torch.equal(pg.cpu(), pc), n
    assert not all(torch.equal(pd.cpu(), pc) for pc, pd in zip(cpu.parameters(), dev.parameters()))
