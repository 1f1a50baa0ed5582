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


def test_deferred_wgrad_grouped_flush_on_gpu():
    """Eligible shapes are queued and issued as one grouped MFMA launch at flush time."""
    torch.manual_seed(0)
    ws, refs, ready = [], [], []
    for out_f, in_f in [(384, 256), (1024, 1024), (256, 520)]:
        w = torch.nn.Parameter(torch.randn(out_f, in_f, device="cuda", dtype=torch.bfloat16))
        w.main_grad = torch.randn(out_f, in_f, device="cuda", dtype=torch.float32)
        w._smdt_grad_ready = lambda p: ready.append(p)
        g = torch.randn(1024, out_f, device="cuda", dtype=torch.bfloat16)
        x = torch.randn(1024, in_f, device="cuda", dtype=torch.bfloat16)
        refs.append(w.main_grad.clone() + g.float().t() @ x.float())
        assert tp._wgrad(w, g, x) is None
        ws.append(w)
    assert ready == [] and len(tp.DEFERRED_WGRAD.items) == 3
    tp.flush_deferred_wgrad()
    assert len(ready) == 3 and not tp.DEFERRED_WGRAD.items
    for w, ref in zip(ws, refs):
        torch.testing.assert_close(w.main_grad, ref, atol=0.5, rtol=1e-2)


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


def test_ddp_main_grads_match_autograd_grads():
    """DDP-owned params: weight (hipBLASLt beta=1), bias and LayerNorm grads are accumulated by the
    kernels straight into fp32 main_grad; they must equal plain autograd .grad of a twin model."""
    from smdt_amd.models.gpt import GPTModel
    from smdt_amd.models.transformer import TransformerConfig
    from smdt_amd.parallel import state as ps
    from smdt_amd.parallel.distributed import DistributedDataParallel
    ps.destroy_model_parallel()
    cfg = TransformerConfig(num_layers=2, hidden_size=256, num_attention_heads=4, padded_vocab_size=512,
                            max_position_embeddings=256, hidden_dropout=0.0, attention_dropout=0.0,
                            params_dtype=torch.bfloat16)
    torch.manual_seed(0)
    a = GPTModel(cfg, device="cuda")
    b = GPTModel(cfg, device="cuda")
    b.load_state_dict(a.state_dict())
    ddp = DistributedDataParallel(a, grad_dtype=torch.float32)
    toks = torch.randint(0, 500, (2, 257), device="cuda")
    for _ in range(2):  # second pass checks accumulation (main_grad += , .grad +=)
        a(toks[:, :-1], labels=toks[:, 1:]).float().mean().backward()
        b(toks[:, :-1], labels=toks[:, 1:]).float().mean().backward()
    ddp.finish_grad_sync()
    pb = dict(b.named_parameters())
    for n, p in a.named_parameters():
        ref = pb[n].grad.float()
        err = (p.main_grad - ref).abs().max().item()
        assert err <= 0.02 * max(1.0, ref.abs().max().item()), (n, err)


@pytest.mark.parametrize("shape", [(4096, 1024, 1024), (1024, 384, 256), (2048, 256, 512)])
@pytest.mark.parametrize("max_splits", [0, 1])
def test_wgrad_mfma_kernel_matches_fp32_reference(shape, max_splits):
    """Hand-written MFMA wgrad (tr-LDS operands, split-K atomics / plain RMW) vs fp32 matmul."""
    from smdt_amd.ops import _ext
    torch.manual_seed(2)
    M, N, K = shape
    g = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    base = torch.randn(N, K, device="cuda", dtype=torch.float32)
    mg = base.clone()
    assert _ext.ext().wgrad_mfma(mg, g, x, max_splits)
    ref = base + g.float().t() @ x.float()
    torch.testing.assert_close(mg, ref, atol=2e-2 * (M ** 0.5), rtol=1e-3)


def test_wgrad_grouped_matches_fp32_reference():
    """One grouped launch over problems of different shapes (incl. partial tiles) == per-problem fp32."""
    from smdt_amd.ops import _ext
    torch.manual_seed(3)
    shapes = [(2048, 1024, 1024), (2048, 384, 256), (1024, 3072, 1024), (4096, 256, 520)]
    mgs, dys, xs, refs = [], [], [], []
    for M, N, K in shapes:
        g = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
        x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        base = torch.randn(N, K, device="cuda", dtype=torch.float32)
        mgs.append(base.clone())
        dys.append(g)
        xs.append(x)
        refs.append(base + g.float().t() @ x.float())
    assert _ext.ext().wgrad_grouped(mgs, dys, xs)
    for (M, _, _), mg, ref in zip(shapes, mgs, refs):
        torch.testing.assert_close(mg, ref, atol=2e-2 * (M ** 0.5), rtol=1e-3)


def test_wgrad_grouped_tail_split_matches_fp32_reference():
    """A grouped launch of 256 whole tiles + a 12-tile tail (partial N and K tiles): the tail is cut
    along m into pieces that add with fp32 atomics; every target must still equal base + dy^T x."""
    from smdt_amd.ops import _ext
    torch.manual_seed(5)
    shapes = [(2048, 1024, 1024)] * 16 + [(2048, 1000, 520)]
    mgs, dys, xs, refs = [], [], [], []
    for M, N, K in shapes:
        g = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
        x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        base = torch.randn(N, K, device="cuda", dtype=torch.float32)
        mgs.append(base.clone())
        dys.append(g)
        xs.append(x)
        refs.append(base + g.float().t() @ x.float())
    assert _ext.ext().wgrad_grouped(mgs, dys, xs)
    for (M, _, _), mg, ref in zip(shapes, mgs, refs):
        torch.testing.assert_close(mg, ref, atol=2e-2 * (M ** 0.5), rtol=1e-3)


@pytest.mark.parametrize("stage", [1, 2])
def test_overlapped_optimizer_step_matches_synchronous(stage, monkeypatch):
    """One DP rank: the per-bucket fused AdamW on a side stream, waited for by the next forward's
    block pre-hooks (parallel/distributed.py overlap_optimizer), gives the synchronous step's
    losses, parameters and optimizer state. The side stream is delayed by ~1 ms before every
    update (SMDT_OPT_STREAM_DELAY), so a missing wait would read stale weights; the tolerance
    only absorbs run-to-run reduction-order noise (atomics in the wgrad tail)."""
    from smdt_amd.models.hf import HFCausalLM
    from smdt_amd.parallel import state as ps
    from smdt_amd.train import zero as Z
    from smdt_amd.train.zero import ZeroEngine
    monkeypatch.setattr(Z, "MIN_BUCKET", 100_000)      # several buckets on this small model
    cfg = dict(model_type="llama", hidden_size=256, num_hidden_layers=3, num_attention_heads=4,
               num_key_value_heads=2, intermediate_size=512, max_position_embeddings=256, vocab_size=512,
               rms_norm_eps=1e-6, rope_theta=10000.0, tie_word_embeddings=False)
    ds = {"bf16": {"enabled": True}, "gradient_accumulation_steps": 2, "gradient_clipping": 1.0,
          "optimizer": {"type": "AdamW", "params": {"lr": 1e-2, "weight_decay": 0.1}},
          "zero_optimization": {"stage": stage, "reduce_bucket_size": 200_000}}
    runs = []
    monkeypatch.setenv("SMDT_OPT_STREAM_DELAY", "2000000")
    for overlap in ("1", "0"):
        monkeypatch.setenv("SMDT_OVERLAP_OPTIMIZER", overlap)
        ps.destroy_model_parallel()
        torch.manual_seed(0)
        m = HFCausalLM(cfg, params_dtype=torch.bfloat16, device="cuda")
        eng = ZeroEngine(m, ds, log=lambda *_: None)
        assert eng.ddp.overlap_optimizer == (overlap == "1") and len(eng.ddp.buckets) > 2
        g = torch.Generator(device="cuda").manual_seed(1)
        losses = []
        for _ in range(6):
            ids = torch.randint(0, 500, (4, 128), device="cuda", generator=g)
            loss, _ = m(ids, labels=ids)
            eng.backward(loss)
            eng.step()
            losses.append(loss.detach().float())
        eng.wait_for_params()
        torch.cuda.synchronize()
        runs.append((torch.stack(losses).cpu(), {n: p.detach().clone() for n, p in m.named_parameters()},
                     eng.optimizer.exp_avg_sq.clone()))
    (l1, p1, v1), (l2, p2, v2) = runs
    # lr 1e-2: one step moves the loss by ~1e-1, so a forward on stale weights would show here
    assert (l1[1:] - l1[:-1]).abs().max() > 1e-2
    torch.testing.assert_close(l1, l2, atol=2e-3, rtol=0)
    for n in p2:
        # elements with near-zero gradients may flip their Adam direction on reduction-order
        # noise (up to lr per step); everything else must agree
        far = ((p1[n].float() - p2[n].float()).abs() > 2e-3 + 1e-2 * p2[n].float().abs()).float().mean().item()
        assert far < 0.01, (n, far)
    assert ((v1 - v2).abs() > 0.05 * v2.abs() + 1e-12).float().mean().item() < 0.01


@pytest.mark.gpu
def test_merged_accumulation_window_wgrad_matches_per_microbatch():
    """ZeRO engine, gradient accumulation 4 on one DP rank: with the merged window
    (parallel/tensor_parallel.DeferredWgrad.hold) every weight's four micro-batch wgrad GEMMs run
    as ONE grouped GEMM over the window's tokens; losses and parameters equal the per-micro-batch
    path (SMDT_WGRAD_MERGE_ACCUM=0) up to fp32 summation order."""
    import os
    from smdt_amd.models.hf import HFCausalLM
    from smdt_amd.parallel import state as ps
    from smdt_amd.parallel import tensor_parallel as tp
    from smdt_amd.train.zero import ZeroEngine
    cfg = dict(model_type="llama", hidden_size=256, num_hidden_layers=2, num_attention_heads=4,
               num_key_value_heads=2, intermediate_size=512, max_position_embeddings=256, vocab_size=512,
               rms_norm_eps=1e-6, rope_theta=10000.0, tie_word_embeddings=False)
    ds = {"bf16": {"enabled": True}, "gradient_accumulation_steps": 4, "gradient_clipping": 1.0,
          "optimizer": {"type": "AdamW", "params": {"lr": 1e-2, "weight_decay": 0.1}},
          "zero_optimization": {"stage": 2}}
    q = tp.DEFERRED_WGRAD
    orig_flush = type(q).flush
    runs = []
    for merge in ("1", "0"):
        os.environ["SMDT_WGRAD_MERGE_ACCUM"] = merge
        segs = []

        def flush(self, _orig=orig_flush, _segs=segs):
            _segs.extend(len(it[2]) for it in self.items)
            return _orig(self)
        type(q).flush = flush
        try:
            ps.destroy_model_parallel()
            torch.manual_seed(0)
            m = HFCausalLM(cfg, params_dtype=torch.bfloat16, device="cuda")
            eng = ZeroEngine(m, ds, log=lambda *_: None)
            g = torch.Generator(device="cuda").manual_seed(1)
            losses = []
            for _ in range(8):          # two optimizer steps
                ids = torch.randint(0, 500, (2, 128), device="cuda", generator=g)
                loss, _ = m(ids, labels=ids)
                eng.backward(loss)
                eng.step()
                losses.append(loss.detach().float())
            eng.wait_for_params()
            torch.cuda.synchronize()
        finally:
            type(q).flush = orig_flush
            os.environ.pop("SMDT_WGRAD_MERGE_ACCUM", None)
            q.hold = False
        runs.append((torch.stack(losses).cpu(), {n: p.detach().float().clone() for n, p in m.named_parameters()},
                     max(segs) if segs else 0))
    (l1, p1, s1), (l2, p2, s2) = runs
    assert s1 == 4 and s2 == 1, (s1, s2)     # merged: 4 micro-batch segments per weight
    torch.testing.assert_close(l1, l2, atol=2e-3, rtol=0)
    for n in p2:
        far = ((p1[n] - p2[n]).abs() > 2e-3 + 1e-2 * p2[n].abs()).float().mean().item()
        assert far < 0.01, (n, far)


def test_sp_norms_write_into_all_gather_slots():
    """Sequence parallelism at TP2 (one process, loopback group): the fused norms write their
    output (forward) and input gradient (backward) into their rank's slot of the ring all-gather
    buffer, so ``ag_ring`` copies nothing; loss and every gradient equal the copying path's."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = "import sys; sys.path[:0] = [%r, %r]; import dist_workers as W; W.sp_gather_slots_worker()" % (
        os.path.join(root, "tests"), root)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300, cwd=root)
    assert r.returncode == 0, r.stderr[-3000:]
    rec = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    # 2 layers: QKV / fc1 forward gathers + proj / fc2 backward gathers + the LM head's = 9 per pass,
    # all in place except the first layer's fc2-less input (none) -> every gather is in place
    assert rec["stats_slots"]["copied"] == 0 and rec["stats_slots"]["in_place"] >= 8, rec
    assert rec["stats_copy"]["in_place"] == 0 and rec["stats_copy"]["copied"] == rec["stats_slots"]["in_place"], rec
    assert rec["same_keys"] and rec["n_grads"] > 10
    assert rec["loss_diff"] == 0.0
    assert rec["grad_max_diff"] < 1e-3, rec


@pytest.mark.parametrize("M", [4300, 4608, 8600, 5000, 4096])
def test_row_split_linear_matches_whole(M):
    """tensor_parallel.linear_rows: token counts just above a multiple of 4096 run as two row
    blocks (hipBLASLt's whole-GEMM kernel for them is slow); the result equals F.linear's."""
    torch.manual_seed(0)
    x = torch.randn(M, 512, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(768, 512, device="cuda", dtype=torch.bfloat16) * 0.05
    b = torch.randn(768, device="cuda", dtype=torch.bfloat16)
    split = tp._row_blocks(M) is not None
    assert split == (M in (4300, 4608, 8600))
    for bias in (None, b):
        ref = x.float() @ w.float().t() + (0 if bias is None else bias.float())
        out = tp.linear_rows(x, w, bias)
        assert out.shape == (M, 768)
        torch.testing.assert_close(out.float(), ref, atol=0.06, rtol=0.02)
    x3 = x.view(M // 4 if M % 4 == 0 else 1, -1, 512) if M % 4 == 0 else x.view(1, M, 512)
    torch.testing.assert_close(tp.linear_rows(x3, w).reshape(M, 768), tp.linear_rows(x, w))


def test_mm_rows_matches_matmul():
    """The NN dgrad form (no W^T) row-splits like linear_rows and equals dY @ W."""
    torch.manual_seed(0)
    w = torch.randn(1024, 2048, device="cuda", dtype=torch.bfloat16) * 0.05
    g = torch.randn(4300, 1024, device="cuda", dtype=torch.bfloat16)
    torch.testing.assert_close(tp.mm_rows(g, w).float(), g.float() @ w.float(), atol=0.08, rtol=0.02)


def test_wgrad_grouped_overwrite_ignores_stale_targets():
    """Grouped wgrad with ``overwrite``: the targets hold garbage (NaN) — the launch STORES
    dy^T x for overwrite problems (no read) and accumulates for the others; a problem whose tiles
    fall into the launch's split tail (atomics) is zeroed first. Bias sums still accumulate."""
    from smdt_amd.ops import _ext
    C = _ext.ext()
    torch.manual_seed(0)
    M = 2048
    shapes = [(768, 512), (1024, 256), (256, 1280)]   # 6 + 4 + 5 = 15 tiles: all in the split tail
    mgs, dys, xs, refs, bias, bref, ow = [], [], [], [], [], [], []
    for i, (n, k) in enumerate(shapes):
        dy = torch.randn(M, n, device="cuda", dtype=torch.bfloat16)
        x = torch.randn(M, k, device="cuda", dtype=torch.bfloat16)
        prod = dy.float().t() @ x.float()
        overwrite = i != 1
        mg = torch.full((n, k), float("nan"), device="cuda") if overwrite else torch.randn(n, k, device="cuda")
        refs.append(prod if overwrite else mg.clone() + prod)
        b = torch.zeros(n, device="cuda")
        bias.append(b)
        bref.append(dy.float().sum(0))
        mgs.append(mg)
        dys.append(dy)
        xs.append(x)
        ow.append(overwrite)
    assert C.wgrad_grouped(mgs, dys, xs, bias, ow)
    for mg, ref in zip(mgs, refs):
        assert torch.isfinite(mg).all()
        torch.testing.assert_close(mg, ref, atol=0.05, rtol=1e-3)
    for b, r in zip(bias, bref):
        torch.testing.assert_close(b, r, atol=0.05, rtol=1e-3)
    # a launch with whole rounds (256 tiles: no tail): the overwrite path proper
    n, k = 4096, 4096                                 # 16 x 16 = 256 tiles
    dy = torch.randn(M, n, device="cuda", dtype=torch.bfloat16)
    x = torch.randn(M, k, device="cuda", dtype=torch.bfloat16)
    mg = torch.full((n, k), float("nan"), device="cuda")
    assert C.wgrad_grouped([mg], [dy], [x], [], [True])
    torch.testing.assert_close(mg, dy.float().t() @ x.float(), atol=0.05, rtol=1e-3)


def test_fused_mlp_waits_for_overlapped_param_gather(monkeypatch):
    """ZeRO-1 with ``overlap_param_gather`` (one emulated DP=2 rank: the parameter all-gather is a
    loopback stand-in on a side stream, delayed ~10 ms so a skipped wait reads stale weights). The
    fused fc1 + bias-GeLU MLP reads fc1 / fc2 weights without calling fc1(x) / fc2(x), so it must
    run their gather-wait pre-hooks itself (models/transformer._gather_wait): its losses equal the
    unfused MLP's, which waits through the modules' own forward pre-hooks."""
    from smdt_amd.models.gpt import GPTModel
    from smdt_amd.models.transformer import TransformerConfig
    from smdt_amd.optim.optimizer import MixedPrecisionAdam
    from smdt_amd.parallel import state as ps
    from smdt_amd.parallel.distributed import DistributedDataParallel
    monkeypatch.setenv("SMDT_LOOPBACK_DELAY_CYCLES", "20000000")
    calls = {"n": 0}
    orig = tp.FusedGeLUMLP.apply

    def counted(*a):
        calls["n"] += 1
        return orig(*a)
    monkeypatch.setattr(tp.FusedGeLUMLP, "apply", counted)
    monkeypatch.setattr(tp, "_fills_chip", lambda rows, n: True)   # test shapes: a few tiles only
    import smdt_amd.models.transformer as T
    real_wait = T._gather_wait
    runs = []
    # third arm, a mutation check of the test itself: the fused MLP WITHOUT its gather waits must
    # read stale weights and move the losses
    for fused, wait in ((True, True), (False, True), (True, False)):
        monkeypatch.setattr(tp, "_FUSED_BIAS_GELU", fused)
        monkeypatch.setattr(T, "_gather_wait", real_wait if wait else (lambda mod, x: None))
        ps.destroy_model_parallel()
        ps.initialize_emulated_tensor_parallel(1, 2)
        torch.manual_seed(0)
        cfg = TransformerConfig(num_layers=2, hidden_size=256, num_attention_heads=4, padded_vocab_size=1024,
                                max_position_embeddings=256, hidden_dropout=0.0, attention_dropout=0.0,
                                params_dtype=torch.bfloat16)
        model = GPTModel(cfg, device="cuda")
        ddp = DistributedDataParallel(model, bucket_size=200_000, use_distributed_optimizer=True,
                                      overlap_param_gather=True)
        assert len(ddp.buckets) > 2
        opt = MixedPrecisionAdam(ddp, lr=1e-2, weight_decay=0.0, clip_grad=1.0)
        g = torch.Generator(device="cuda").manual_seed(1)
        tokens = torch.randint(0, 1000, (4, 257), device="cuda", generator=g)
        losses = []
        for _ in range(4):
            ddp.zero_grad_buffer()
            loss = ddp(tokens[:, :-1], None, None, labels=tokens[:, 1:]).float().mean()
            loss.backward()
            ddp.finish_grad_sync()
            opt.step()
            losses.append(loss.detach())
        ddp.wait_param_gather()
        torch.cuda.synchronize()
        runs.append(torch.stack(losses).cpu())
        if fused:
            assert calls["n"] >= 4 * cfg.num_layers, calls      # the fused MLP really ran
    ps.destroy_model_parallel()
    a, b, stale = runs
    assert (a[1:] - a[:-1]).abs().max() > 1e-2          # steps move the loss: stale weights would show
    torch.testing.assert_close(a, b, atol=2e-2, rtol=0)
    assert (stale - b).abs().max() > 5 * (a - b).abs().max(), (a, b, stale)


@pytest.mark.parametrize("stream", [False, True])
def test_w_fillers_match_grouped_flush_on_gpu(monkeypatch, stream):
    """One emulated tp2 + SP rank, split backward over 3 micro-batches (the zero-bubble stage's W
    grouping), TP exchanges on the paced link stand-in so they hold CUs: with SMDT_W_FILL the W
    GEMMs run as fillers inside the exchange waits (single items, tail split sized to the free
    CUs, fp32 atomics) instead of one grouped flush per pass — on the compute stream, or on a
    filler stream of their own (``stream``: joined at each pass end, readiness reported after the
    join). The fp32 main_grad buffer and the losses match the flush run, and fillers really ran."""
    from smdt_amd.models.gpt import GPTModel
    from smdt_amd.models.transformer import TransformerConfig
    from smdt_amd.parallel import state as ps
    from smdt_amd.parallel.distributed import DistributedDataParallel as DDP
    from smdt_amd.train.schedules import forward_backward_no_pipelining
    monkeypatch.setenv("SMDT_LINK_STANDIN", "256:32")
    monkeypatch.setattr(tp, "_FILL_STREAM_ON", stream)
    out = []
    for fill in (False, True):
        monkeypatch.setattr(tp, "W_FILL", fill)
        tp.DEFERRED_WGRAD.stats.pop("fills", None)
        ps.destroy_model_parallel()
        ps.initialize_emulated_tensor_parallel(2, 1)
        try:
            cfg = TransformerConfig(num_layers=2, hidden_size=256, num_attention_heads=4, padded_vocab_size=1024,
                                    max_position_embeddings=256, hidden_dropout=0.0, attention_dropout=0.0,
                                    params_dtype=torch.bfloat16, sequence_parallel=True, seed=7)
            model = GPTModel(cfg, device="cuda")
            ddp = DDP(model, grad_dtype=torch.float32)
            g = torch.Generator(device="cuda").manual_seed(13)
            t = torch.randint(0, 1000, (6, 257), device="cuda", generator=g)
            data = iter([(t[2 * i:2 * i + 2, :-1], t[2 * i:2 * i + 2, 1:]) for i in range(3)])

            def fstep(di, m):
                x, y = next(di)
                o = m(x, None, None, labels=y)
                return o, (lambda z: (z.float().mean(), {"loss": z.detach().float().mean()}))
            ddp.zero_grad_buffer()
            losses = forward_backward_no_pipelining(fstep, data, ddp, 3, split_backward=True)
            ddp.finish_grad_sync()
            torch.cuda.synchronize()
            out.append((torch.stack([d["loss"] for d in losses]).cpu(), ddp.grad_data.clone(),
                        tp.DEFERRED_WGRAD.stats.get("fills", 0)))
        finally:
            ps.destroy_model_parallel()
    (l0, g0, f0), (l1, g1, f1) = out
    assert f0 == 0 and f1 > 0
    torch.testing.assert_close(l1, l0, atol=1e-4, rtol=0)
    scale = g0.abs().max().item()
    assert scale > 0 and (g1 - g0).abs().max().item() <= 1e-3 * scale


@pytest.mark.parametrize("sub,pieces", [(0, 1), (2, 1), (0, 2)])
def test_direct_engine_standin_matches_ring_emulation(monkeypatch, sub, pieces):
    """One emulated tp4 + SP rank with SMDT_LINK_STANDIN=direct: the SP exchanges go through
    ``TpDirect`` (per-piece handles) over the paced stand-in of the direct engine
    (comm/loopback.PacedDirectEngine) instead of the loopback ring. The stand-in's values are the
    loopback ring's (gather = own shard in every slot, reduce-scatter = sum of this rank's
    partials), so losses and the fp32 gradient buffer agree with the ring run to bf16 add-order
    rounding; with W fillers on, fillers ran inside the direct waits. ``sub`` = 2: the direct run
    with the sub-batch interleave (whole-chunk exchanges started by ``ag_start`` / left in flight
    by ``rs_ring``). ``pieces`` = 1: whole chunks (the default); 2: row pieces (per-piece handles,
    per-peer GEMMs as each piece lands)."""
    import smdt_amd.models.transformer as T
    from smdt_amd.comm import tp_direct
    monkeypatch.setattr(tp_direct, "PIECES", pieces)
    from smdt_amd.models.gpt import GPTModel
    from smdt_amd.models.transformer import TransformerConfig
    from smdt_amd.parallel import state as ps
    from smdt_amd.parallel.distributed import DistributedDataParallel as DDP
    from smdt_amd.train.schedules import forward_backward_no_pipelining
    out = []
    for standin in ("", "direct:64:32"):
        monkeypatch.setenv("SMDT_LINK_STANDIN", standin)
        monkeypatch.setattr(tp, "W_FILL", bool(standin))
        monkeypatch.setattr(T, "_SUBBATCH", sub if standin else 0)
        tp.DEFERRED_WGRAD.stats.pop("fills", None)
        started = tp.SPLIT_STATS["ag_started"]
        ps.destroy_model_parallel()
        st = ps.initialize_emulated_tensor_parallel(4, 1)
        try:
            td = getattr(st, "tp_direct", None)
            assert (td is not None) == bool(standin)
            cfg = TransformerConfig(num_layers=2, hidden_size=256, num_attention_heads=4, padded_vocab_size=1024,
                                    max_position_embeddings=256, hidden_dropout=0.0, attention_dropout=0.0,
                                    params_dtype=torch.bfloat16, sequence_parallel=True, seed=7)
            model = GPTModel(cfg, device="cuda")
            ddp = DDP(model, grad_dtype=torch.float32)
            g = torch.Generator(device="cuda").manual_seed(13)
            t = torch.randint(0, 1000, (6, 257), device="cuda", generator=g)
            data = iter([(t[2 * i:2 * i + 2, :-1], t[2 * i:2 * i + 2, 1:]) for i in range(3)])

            def fstep(di, m):
                x, y = next(di)
                o = m(x, None, None, labels=y)
                return o, (lambda z: (z.float().mean(), {"loss": z.detach().float().mean()}))
            ddp.zero_grad_buffer()
            losses = forward_backward_no_pipelining(fstep, data, ddp, 3, split_backward=True)
            ddp.finish_grad_sync()
            torch.cuda.synchronize()
            out.append((torch.stack([d["loss"] for d in losses]).cpu(), ddp.grad_data.clone(),
                        tp.DEFERRED_WGRAD.stats.get("fills", 0), td.pieces_issued if td else 0))
            assert (tp.SPLIT_STATS["ag_started"] > started) == bool(standin and sub)
        finally:
            tp.DEFERRED_WGRAD.merge_repeats = False
            ps.destroy_model_parallel()
    (l0, g0, _, p0), (l1, g1, f1, p1) = out
    assert p0 == 0 and p1 > 0 and f1 > 0
    torch.testing.assert_close(l1, l0, atol=2e-2, rtol=0)
    scale = g0.abs().max().item()
    assert scale > 0 and (g1 - g0).abs().max().item() <= 3e-2 * scale
