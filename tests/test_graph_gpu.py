"""HIP-graph capture of a whole data-parallel training step.

One MI355X, one process as rank 0 of an emulated 8-rank DP job (loopback DP group,
comm/loopback.py: the reduce-scatter / all-gather stand-ins run on the group's side stream as an
RCCL collective would). The step — forward, backward with the framework DDP's bucketed gradient
reductions, the hand-written fused Adam with its device-side step count (optim.hip
``adam_capturable``), and for ZeRO-1 the parameter all-gather — is captured once and replayed;
parameters after the replays equal the same steps run eagerly.
"""
import pytest
import torch
import torch.nn as nn

pytestmark = pytest.mark.gpu


def _model():
    torch.manual_seed(3)
    return nn.Sequential(nn.Conv2d(3, 16, 3, padding=1), nn.ReLU(), nn.AdaptiveAvgPool2d(4), nn.Flatten(),
                         nn.Linear(256, 64), nn.ReLU(), nn.Linear(64, 10)).cuda()


def _run(zero, graph, steps=4):
    from smdt_amd.optim.optimizer import MixedPrecisionAdam
    from smdt_amd.parallel import state as ps
    from smdt_amd.parallel.distributed import DistributedDataParallel as DDP
    ps.destroy_model_parallel()
    ps.initialize_emulated_tensor_parallel(1, 8)
    ddp = DDP(_model(), torch_compat=True, bucket_size=4096, use_distributed_optimizer=zero)
    assert ddp.dp == 8
    opt = MixedPrecisionAdam(ddp, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, adamw=False,
                             capturable=True)
    g = torch.Generator(device="cuda").manual_seed(7)
    x = torch.randn(16, 3, 8, 8, device="cuda", generator=g)
    y = torch.randint(0, 10, (16,), device="cuda", generator=g)
    crit = nn.CrossEntropyLoss()

    def step():
        loss = crit(ddp(x), y)
        loss.backward()
        opt.step()
        ddp.wait_param_gather()            # ZeRO-1: the all-gather completes inside the step
        return loss

    if not graph:
        losses = [step().item() for _ in range(steps)]
    else:
        step()                             # one eager step (algorithm selection, buffers)
        torch.cuda.synchronize()
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr):
            static_loss = step()
        losses = [None]                    # (the capture itself ran no kernels)
        for _ in range(steps - 1):
            gr.replay()
            losses.append(static_loss.item())
    torch.cuda.synchronize()
    params = [p.detach().clone() for p in ddp.module.parameters()]
    st = opt.state_dict()["step"]
    ps.destroy_model_parallel()
    return losses, params, st


@pytest.mark.parametrize("zero", [False, True])
def test_captured_emulated_dp8_step_equals_eager(zero):
    le, pe, se = _run(zero, graph=False)
    lg, pg, sg = _run(zero, graph=True)
    assert se == sg == 4                   # the device step count advanced on every replay
    for a, b in zip(le[1:], lg[1:]):
        assert abs(a - b) <= 1e-5 * max(1.0, abs(a)), (le, lg)
    for a, b in zip(pe, pg):
        torch.testing.assert_close(b, a, rtol=1e-5, atol=1e-6)


def _gpt_emulated_tp_run(graph, steps=3, sp=True):
    """One process as TP rank 0 of a tp2 (+SP) GPT (loopback TP group): eager steps, or one eager
    step then a captured step replayed. Dropout off, so eager and replayed steps see the same
    math; returns per-step losses and the fp32 main_grad buffer after the last step."""
    import os
    from smdt_amd.models.gpt import GPTModel
    from smdt_amd.models.transformer import TransformerConfig
    from smdt_amd.optim.optimizer import MixedPrecisionAdam
    from smdt_amd.parallel import state as ps
    from smdt_amd.parallel.distributed import DistributedDataParallel as DDP
    from smdt_amd.train.schedules import get_forward_backward_func
    ps.destroy_model_parallel()
    ps.initialize_emulated_tensor_parallel(2, 1)
    cfg = TransformerConfig(num_layers=2, hidden_size=256, num_attention_heads=4, padded_vocab_size=1024,
                            max_position_embeddings=256, hidden_dropout=0.0, attention_dropout=0.0,
                            params_dtype=torch.bfloat16, sequence_parallel=sp, seed=5)
    model = GPTModel(cfg, device="cuda")
    ddp = DDP(model, grad_dtype=torch.float32)
    opt = MixedPrecisionAdam(ddp, lr=1e-3, weight_decay=0.01, clip_grad=1.0, capturable=True)
    g = torch.Generator(device="cuda").manual_seed(11)
    toks = [torch.randint(0, 1000, (2, 129), device="cuda", generator=g) for _ in range(2)]
    fb = get_forward_backward_func()
    shape = (64 if sp else 128, 2, 256)

    def fstep(it, m):
        t = next(it)
        out = m(t[:, :-1], None, None, labels=t[:, 1:])
        return out, (lambda o: (o.float().mean(), {"lm loss": o.float().mean().detach()}))

    def step():
        ddp.zero_grad_buffer()
        r = fb(fstep, iter(toks), ddp, 2, tensor_shape=shape, dtype=torch.bfloat16)
        ddp.finish_grad_sync()
        opt.step()
        return torch.stack([d["lm loss"] for d in r])

    losses, mg = [], None
    if not graph:
        for _ in range(steps):
            losses.append(step().clone())
            if len(losses) == steps - 1:
                mg = ddp.grad_data.clone()
    else:
        losses.append(step().clone())
        torch.cuda.synchronize()
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr):
            sl = step()
        for i in range(steps - 1):
            gr.replay()
            losses.append(sl.clone())
            if len(losses) == steps - 1:
                mg = ddp.grad_data.clone()
    torch.cuda.synchronize()
    ps.destroy_model_parallel()
    return torch.stack(losses).cpu(), mg.cpu()


@pytest.mark.parametrize("sp", [True, False])
def test_captured_emulated_tp2_gpt_step_equals_eager(sp):
    """A whole GPT training step of one emulated tp2 rank (ring collective-matmul exchanges as
    loopback copies, two micro-batches, DDP sync, capturable fused Adam) captured once and
    replayed: per-step losses and the accumulated fp32 main_grad equal the eager steps."""
    le, ge = _gpt_emulated_tp_run(False, sp=sp)
    lg, gg = _gpt_emulated_tp_run(True, sp=sp)
    torch.testing.assert_close(lg, le, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(gg, ge, rtol=1e-4, atol=1e-6)


def test_subbatch_interleave_emulated_tp2_step_matches_default(monkeypatch):
    """The sub-batch interleave (SMDT_SP_SUBBATCH=2) on the GPU kernel path of one emulated tp2 +
    SP rank: the fused norms return views of the all-gather buffers that ``tp.ag_start`` fills
    early, the halves' reduce-scatters complete in ``tp.rs_finish``. Same losses and fp32
    main_grad as the default layer loop up to bf16 GEMM-shape rounding (one GEMM over both
    chunks instead of two)."""
    import smdt_amd.models.transformer as T
    from smdt_amd.parallel import tensor_parallel as TPm
    le, ge = _gpt_emulated_tp_run(False, sp=True)
    monkeypatch.setattr(T, "_SUBBATCH", 2)
    before = dict(TPm.SPLIT_STATS)
    try:
        ls, gs = _gpt_emulated_tp_run(False, sp=True)
    finally:
        TPm.DEFERRED_WGRAD.merge_repeats = False
    assert TPm.SPLIT_STATS["ag_started"] > before["ag_started"]
    torch.testing.assert_close(ls, le, rtol=2e-2, atol=2e-2)
    assert (gs - ge).abs().max() <= 3e-2 * ge.abs().max()


def test_reduce_scatter_combine_in_norms_matches_plain_combine(monkeypatch):
    """One emulated tp2 + SP rank on the kernel path: with the ring reduce-scatters' combines left
    to the fused norms (forward: the norm reads x + x2; backward: the norm backward reads dy +
    dy2) the losses and fp32 main_grad equal the plain separate-add path up to bf16 rounding, and
    both deferrals really ran."""
    from smdt_amd.parallel import tensor_parallel as TPm
    monkeypatch.setattr(TPm, "_DEFER_RS_ADD", False)
    lo, go = _gpt_emulated_tp_run(False, sp=True)
    monkeypatch.setattr(TPm, "_DEFER_RS_ADD", True)
    before = dict(TPm.SPLIT_STATS)
    ld, gd = _gpt_emulated_tp_run(False, sp=True)
    assert TPm.SPLIT_STATS["rs_add_to_norm"] > before["rs_add_to_norm"]
    assert TPm.SPLIT_STATS["bwd_add_to_norm"] > before["bwd_add_to_norm"]
    torch.testing.assert_close(ld, lo, rtol=1e-2, atol=1e-2)
    assert (gd - go).abs().max() <= 2e-2 * go.abs().max()


def test_bench_graph_mode_captures(tmp_path):
    """bench.py --graph 1 on an emulated tp2 last-stage rank reports a captured HIP graph."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, os.path.join(root, "bench.py"), "--graph", "1", "--emulate-tp", "2", "--emulate-last-stage",
           "--num-layers", "2", "--hidden-size", "256", "--num-attention-heads", "4", "--seq-length", "256",
           "--micro-batch-size", "2", "--grad-accum", "2", "--steps", "3", "--warmup", "2", "--tunableop", "0",
           "--phase-probe", "0"]
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=str(tmp_path), env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    rec = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert rec["config"]["hip_graph"] == "captured", rec["config"]["hip_graph"]
