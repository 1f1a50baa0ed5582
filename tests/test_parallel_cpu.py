"""Parallel-equivalence tests on CPU / gloo: TP, SP, PP and DP/ZeRO runs must
reproduce the single-process run on the same seed and data."""
import pytest
import torch

import dist_workers as W
from _dist import run_workers

pytestmark = pytest.mark.slow


def _close(a, b, tol=2e-4):
    torch.testing.assert_close(a, b, atol=tol, rtol=tol)


def _check_tp_grads(ref, grads, meta, tp):
    r = meta["tp_rank"]
    off = meta["layer_offset"]
    for name, g in grads.items():
        rname = name
        if name.startswith("decoder.layers."):
            parts = name.split(".")
            parts[2] = str(int(parts[2]) + off)
            rname = ".".join(parts)
        if name == "output_weight":
            rname = "embedding.weight"
        full = ref[rname]
        if full.shape == g.shape:
            _close(g, full)
            continue
        # sharded parameter: find the split dimension
        if "qkv.weight" in name or "qkv.bias" in name:
            h = full.shape[0] // 3
            parts = [full[i * h:(i + 1) * h].chunk(tp, 0)[r] for i in range(3)]
            _close(g, torch.cat(parts, 0))
        elif full.shape[0] != g.shape[0]:
            _close(g, full.chunk(tp, 0)[r])
        else:
            _close(g, full.chunk(tp, 1)[r])


@pytest.mark.parametrize("tp,sp", [(2, False), (2, True), (4, True), (4, False)])
def test_tensor_parallel_matches_single_rank(tp, sp):
    """tp 4 + SP exercises the multi-step collective-matmul rings (send next / recv prev); tp 2 + SP
    the forward reduce-scatters whose combine the consuming fused norm does (x2 summand)."""
    ref_loss, ref = W.gpt_reference()
    outs = run_workers(W.gpt_tp_worker, tp, tp, 1, sp)
    for loss, grads, meta in outs:
        _close(loss, ref_loss)
        _check_tp_grads(ref, grads, meta, tp)
        # tp2 + SP: the forward reduce-scatters left their combine to the consuming norms
        assert (meta["split"]["rs_add_to_norm"] > 0) == (sp and tp == 2)


@pytest.mark.parametrize("tp,pieces", [(4, 1), (4, 2), (2, 4)])
def test_direct_tp_exchange_pieces_match_single_rank(tp, pieces):
    """TP + SP with every sequence-parallel exchange through ``TpDirect`` in row pieces (a CPU
    stand-in of the xGMI engine's piece calls over Gloo): the all-gather callers get row ranges
    (lo, rows) piece by piece, the reduce-scatter callers write their partials straight into the
    engine's input (``partial_fn(lo, rows, out)``) — column / row SP linears, both directions.
    Loss and every gradient equal the single-rank model's."""
    ref_loss, ref = W.gpt_reference()
    outs = run_workers(W.gpt_tp_worker, tp, tp, 1, True, None, None, pieces)
    for loss, grads, meta in outs:
        _close(loss, ref_loss)
        _check_tp_grads(ref, grads, meta, tp)
        assert meta["direct_calls"] > 0 and meta["direct_pieces"] == pieces * meta["direct_calls"]


@pytest.mark.parametrize("pp", [1, 2])
def test_direct_tp4_subbatch_interleave_matches_single_rank(pp):
    """tp4 + SP over ``TpDirect`` (CPU stand-in engine) with the sub-batch interleave
    (SMDT_SP_SUBBATCH=2): each half's whole-chunk gathers are started by ``ag_start`` and its
    reduce-scatters left in flight (``TpDirect.start_all_gather`` / ``start_reduce_scatter``)
    while the other half's phase runs. Loss and every gradient equal the single-rank model's, and
    the interleave really ran over the engine."""
    ref_loss, ref = W.gpt_reference()
    outs = run_workers(W.gpt_tp_worker, 4 * pp, 4, pp, True, None, None, 2, 2)
    for loss, grads, meta in outs:
        _check_tp_grads(ref, grads, meta, 4)
        assert meta["split"]["ag_started"] > 0 and meta["split"]["rs_deferred"] > 0
        assert meta["direct_calls"] > 0
    last = [o for o in outs if o[2]["pp_rank"] == pp - 1][0]
    torch.testing.assert_close(last[0].view(-1), ref_loss.view(-1), atol=2e-4, rtol=2e-4)


@pytest.mark.parametrize("pp", [1, 2])
def test_ring_pieces_match_single_rank(pp):
    """tp2 + SP with every 2-rank ring exchange in 2 row pieces (SMDT_RING_PIECES=2: the peer
    chunk's GEMM per landed piece, the reduce-scatter's partial sent piece by piece): loss and
    every gradient equal the single-rank model's, and the pieces really ran."""
    ref_loss, ref = W.gpt_reference()
    outs = run_workers(W.gpt_tp_worker, 2 * pp, 2, pp, True, None, None, 0, 0, 2)
    for loss, grads, meta in outs:
        _check_tp_grads(ref, grads, meta, 2)
        assert meta["split"].get("ring_pieces", 0) > 0
    last = [o for o in outs if o[2]["pp_rank"] == pp - 1][0]
    torch.testing.assert_close(last[0].view(-1), ref_loss.view(-1), atol=2e-4, rtol=2e-4)


@pytest.mark.parametrize("pp", [1, 2])
def test_subbatch_interleave_matches_single_rank(pp):
    """tp2 + SP with the two batch halves of every micro-batch interleaved phase by phase
    (SMDT_SP_SUBBATCH=2: one half's all-gather / reduce-scatter in flight while the other half's
    layer phase runs, ``tp.ag_start`` / ``rs_finish``): loss and every gradient equal the
    single-rank model's, and the interleave really ran (4 started exchanges per layer, half and
    micro-batch)."""
    ref_loss, ref = W.gpt_reference()
    outs = run_workers(W.gpt_tp_worker, 2 * pp, 2, pp, True, None, None, 0, 2)
    for loss, grads, meta in outs:
        _check_tp_grads(ref, grads, meta, 2)
        assert meta["split"]["ag_started"] > 0 and meta["split"]["ag_started"] == meta["split"]["rs_deferred"]
    last = [o for o in outs if o[2]["pp_rank"] == pp - 1][0]
    torch.testing.assert_close(last[0].view(-1), ref_loss.view(-1), atol=2e-4, rtol=2e-4)


def test_ag_start_on_a_gather_slot_view():
    """The sub-batch interleave's early all-gather on a norm-style output that is a view of the
    gather buffer (multi-output autograd node, as the fused norm returns on the GPU): forward and
    input gradient equal the plain ring's, and autograd does not refuse the buffer write (the
    loopback rank's exchange is an in-place copy into the buffer: refused without the ``.data``
    alias, checked by mutation)."""
    for world, emulate in ((2, False), (1, True)):     # Gloo pair; loopback (in-place copy) rank
        for res in run_workers(W.ag_start_view_worker, world, emulate):
            for a, b in zip(res["ring"], res["started"]):
                torch.testing.assert_close(a, b)


@pytest.mark.parametrize("over", [None, {"num_layers": 3, "decoder_last_pipeline_num_layers": 1}])
def test_pipeline_parallel_matches_single_rank(over):
    """pp = 2, uniform split and the uneven split bench.py uses to balance the LM head (first stage
    2 layers, last stage 1 layer + head)."""
    ref_loss, ref = W.gpt_reference(cfg_over=over)
    outs = run_workers(W.gpt_tp_worker, 2, 1, 2, False, over)
    last = outs[1]
    # last stage sees the per-token losses of both micro-batches
    torch.testing.assert_close(last[0].view(-1), ref_loss.view(-1), atol=2e-4, rtol=2e-4)
    for loss, grads, meta in outs:
        # micro-batch losses are averaged per micro-batch: scale matches full-batch mean
        _check_tp_grads({k: v for k, v in ref.items()}, grads, meta, 1)


@pytest.mark.parametrize("sp,p2p", [(True, None), (False, None), (False, {"overlap": True}),
                                    (False, {"scatter_gather": False, "deallocate_outputs": False})])
def test_tp2_pp2_dp1_world4(sp, p2p):
    """Without SP the p2p activations are TP-replicated: scatter-gather sends 1/tp of each and
    all-gathers on receipt; --overlap-p2p-communication defers every receive wait to its consumer."""
    ref_loss, ref = W.gpt_reference()
    outs = run_workers(W.gpt_tp_worker, 4, 2, 2, sp, None, p2p)
    for loss, grads, meta in outs:
        _check_tp_grads(ref, grads, meta, 2)
    last = [o for o in outs if o[2]["pp_rank"] == 1][0]
    torch.testing.assert_close(last[0].view(-1), ref_loss.view(-1), atol=2e-4, rtol=2e-4)


@pytest.mark.parametrize("zero,overlap_pg,defer", [(False, False, False), (True, False, False), (True, True, False),
                                                   (False, False, True), (True, True, True)])
def test_data_parallel_and_zero_match_single_process(zero, overlap_pg, defer):
    ref, ref_g = W.single_train()
    outs = run_workers(W.ddp_worker, 2, zero, 3, overlap_pg, defer)
    for params, grads in outs:
        for n, g in grads.items():   # reduced gradients: the reference combines in the same order
            torch.testing.assert_close(g, ref_g[n], atol=0, rtol=0)
        for n, p in params.items():  # Adam at eps 1e-8: equal gradients, so no flipped step signs
            torch.testing.assert_close(p, ref[n], atol=1e-5, rtol=1e-5)


@pytest.mark.parametrize("nmb,p2p", [(2, None), (4, None), (2, {"overlap": True}), (4, {"overlap": True})])
def test_interleaved_pipeline_matches_single_rank(nmb, p2p):
    """pp=2 x vpp=2 (4 layers, chunk c of rank r = global stage 2c + r); nmb == pp exercises the
    all-warm-up path, nmb == 2 pp the steady 1F1B phase."""
    ref_loss, ref = W.gpt_reference(cfg_over={"num_layers": 4})
    outs = run_workers(W.gpt_vpp_worker, 2, nmb, p2p)
    torch.testing.assert_close(outs[1][0].view(-1), ref_loss.view(-1), atol=2e-4, rtol=2e-4)
    seen = set()
    for _, grads in outs:
        for n, g in grads.items():
            _close(g, ref[n])
            seen.add(n)
    assert seen == set(ref), set(ref) ^ seen


def test_deferred_wgrad_queue_semantics(monkeypatch):
    """DeferredWgrad (CPU fallback): ready only at flush, duplicate target flushes first (order kept),
    threshold flush, and an in-place write into a queued operand is caught."""
    from smdt_amd.parallel import tensor_parallel as tp
    q = tp.DeferredWgrad()
    q.allow_cpu = True
    q.flush_tiles = 3
    monkeypatch.setattr(tp, "DEFERRED_WGRAD", q)
    torch.manual_seed(0)
    ready = []

    def mk(o, i):
        w = torch.nn.Parameter(torch.randn(o, i))
        w.main_grad = torch.zeros(o, i)
        w._smdt_grad_ready = lambda p: ready.append(p)
        return w

    a, b = mk(16, 8), mk(8, 8)
    g1, x1 = torch.randn(64, 16), torch.randn(64, 8)
    assert tp._wgrad(a, g1, x1) is None and not ready
    g2, x2 = torch.randn(64, 8), torch.randn(64, 8)
    tp._wgrad(b, g2, x2)
    assert not ready and len(q.items) == 2
    g3, x3 = torch.randn(64, 16), torch.randn(64, 8)
    tp._wgrad(a, g3, x3)            # same target again: the first two are flushed first
    assert ready == [a, b] and len(q.items) == 1
    q.flush()
    assert ready == [a, b, a]
    torch.testing.assert_close(a.main_grad, g1.t() @ x1 + g3.t() @ x3)
    torch.testing.assert_close(b.main_grad, g2.t() @ x2)
    # threshold: 1024-wide weights are 4 x 4 = 16 tiles >= 3 -> immediate flush
    c = mk(1024, 1024)
    tp._wgrad(c, torch.randn(32, 1024), torch.randn(32, 1024))
    assert ready[-1] is c and not q.items
    # in-place modification of a queued operand is an error, not a silent wrong gradient
    g4 = torch.randn(64, 16)
    tp._wgrad(a, g4, torch.randn(64, 8))
    g4.mul_(2)
    with pytest.raises(RuntimeError, match="modified in place"):
        q.flush()
    # ineligible shapes (tokens not a multiple of 32) run immediately
    tp._wgrad(b, torch.randn(33, 8), torch.randn(33, 8))
    assert ready[-1] is b and not q.items


def test_deferred_wgrad_accumulation_window_merges(monkeypatch):
    """DeferredWgrad.hold (the ZeRO engine's gradient-accumulation window): nothing flushes during
    the window, every weight's micro-batch GEMMs merge into ONE product over the concatenated
    tokens with ONE readiness report in the boundary pass, and the result equals the per-micro-
    batch sum."""
    from smdt_amd.parallel import tensor_parallel as tp
    q = tp.DeferredWgrad()
    q.allow_cpu = True
    q.flush_tiles = 1                 # would flush after every push outside a window
    monkeypatch.setattr(tp, "DEFERRED_WGRAD", q)
    torch.manual_seed(1)
    ready = []
    w = torch.nn.Parameter(torch.randn(1024, 64))
    w.main_grad = torch.zeros(1024, 64)
    w._smdt_grad_ready = lambda p: ready.append(p)
    gs = [torch.randn(32 * (i + 1), 1024) for i in range(4)]      # micro-batches of 32 .. 128 tokens
    xs = [torch.randn(32 * (i + 1), 64) for i in range(4)]
    calls = []
    orig_cat = torch.cat
    monkeypatch.setattr(torch, "cat", lambda t, *a, **k: calls.append(len(t)) or orig_cat(t, *a, **k))
    q.hold = True
    for g, x in zip(gs[:3], xs[:3]):
        tp._wgrad(w, g, x)
    assert not ready and len(q.items) == 1 and len(q.items[0][2]) == 3
    q.hold = False                   # the boundary micro-batch
    tp._wgrad(w, gs[3], xs[3])       # merges, then the size threshold flushes the window at once
    assert ready == [w] and not q.items and calls == [4, 4]
    ref = sum(g.t() @ x for g, x in zip(gs, xs))
    torch.testing.assert_close(w.main_grad, ref, atol=2e-4, rtol=1e-4)   # fp32 summation order


def test_accumulation_window_gate(monkeypatch):
    """accumulation_window_ok: the ZeRO engine's default (on) and the Megatron schedule's (off,
    profiles/r3_l4l/), SMDT_WGRAD_MERGE_ACCUM forcing either way, and the structural vetoes
    (ZeRO-3 partitioner, stage 2 without its in-place single-rank store, queue disabled)."""
    from types import SimpleNamespace as NS
    from smdt_amd.parallel import tensor_parallel as tp
    q = tp.DeferredWgrad()
    monkeypatch.setattr(q, "enabled", True, raising=False)
    monkeypatch.setattr(tp, "DEFERRED_WGRAD", q)
    monkeypatch.delenv("SMDT_WGRAD_MERGE_ACCUM", raising=False)
    plain = NS(zero_stage=1)
    assert tp.accumulation_window_ok([plain]) is True
    assert tp.accumulation_window_ok([plain], default=False) is False
    monkeypatch.setenv("SMDT_WGRAD_MERGE_ACCUM", "1")
    assert tp.accumulation_window_ok([plain], default=False) is True
    assert tp.accumulation_window_ok([NS(zero_stage=3, zero3=object())]) is False
    assert tp.accumulation_window_ok([NS(zero_stage=2)]) is False
    assert tp.accumulation_window_ok([NS(zero_stage=2, _direct=True)]) is True
    monkeypatch.setenv("SMDT_WGRAD_MERGE_ACCUM", "0")
    assert tp.accumulation_window_ok([plain]) is False
    monkeypatch.delenv("SMDT_WGRAD_MERGE_ACCUM")
    q.enabled = False
    assert tp.accumulation_window_ok([plain]) is False


@pytest.mark.parametrize("cp,nh,nkv", [(2, 4, 4), (4, 8, 8), (4, 8, 2), (2, 6, 3)])
def test_ulysses_context_parallel_matches_full_attention(cp, nh, nkv):
    """P10 stretch: Ulysses all-to-all context parallelism over gloo reproduces full-sequence causal
    attention (forward and q/k/v gradients, MHA and GQA) on every rank's sequence chunk."""
    from smdt_amd.ops.functional import attention_ref
    s, b, d = 32, 2, 16
    res = run_workers(W.ulysses_worker, cp, nh, nkv, s, b, d)
    g = torch.Generator().manual_seed(7)
    q = torch.randn(s, b, nh, d, generator=g, dtype=torch.float64).requires_grad_(True)
    k = torch.randn(s, b, nkv, d, generator=g, dtype=torch.float64).requires_grad_(True)
    v = torch.randn(s, b, nkv, d, generator=g, dtype=torch.float64).requires_grad_(True)
    dy = torch.randn(s, b, nh, d, generator=g, dtype=torch.float64)
    ref = attention_ref(q.transpose(0, 1), k.transpose(0, 1), v.transpose(0, 1), d ** -0.5, True, 0.0, None)
    ref = ref.transpose(0, 1)
    ref.backward(dy)
    for r, (out, dq, dk, dv) in enumerate(res):
        for got, full in ((out, ref.detach()), (dq, q.grad), (dk, k.grad), (dv, v.grad)):
            _close(got, full.chunk(cp, 0)[r], tol=1e-9)


@pytest.mark.parametrize("tp,cp,sp,over,ddp", [
    (1, 2, False, None, False),
    (1, 4, False, None, True),                                            # cp4 through the DDP wrapper
    (2, 2, True, None, True),                                             # tp2 x cp2 + SP (world 4)
    (1, 2, False, {"position_embedding_type": "rope", "num_query_groups": 2}, False),   # RoPE + GQA
])
def test_gpt_context_parallel_matches_single_rank(tp, cp, sp, over, ddp):
    """P10 / §5.7: --context-parallel-size wired through the model. Each CP rank feeds its sequence
    chunk (positions offset by cp_rank), attention re-shards heads by all-to-all, and gradients
    averaged over dp x cp equal the single-process full-sequence gradients."""
    ref_loss, ref = W.gpt_reference(cfg_over=over)
    outs = run_workers(W.gpt_cp_worker, tp * cp, tp, cp, sp, over, ddp)
    for loss, grads, meta in outs:
        assert len(meta["cp_ranks"]) == cp and len(meta["dp_cp_ranks"]) == cp
        _close(loss, ref_loss.chunk(cp, 1)[meta["cp_rank"]])
        _check_tp_grads(ref, grads, meta, tp)


@pytest.mark.parametrize("async_save", [False, True])
def test_context_parallel_rng_resume(tmp_path, async_save):
    """every CP rank restores its own (shifted) RNG streams from a checkpoint, so dropout
    masks after a resume match an uninterrupted run and stay decorrelated across CP ranks (also
    with --async-save: per-rank background writers, the tracker after both finished)."""
    outs = run_workers(W.cp_rng_resume_worker, 2, str(tmp_path), async_save)
    assert sorted(o["cp_rank"] for o in outs) == [0, 1]
    assert all(o["same"] for o in outs), outs
    assert outs[0]["mask"] != outs[1]["mask"]


@pytest.mark.parametrize("world,tp,pp,nmb,zero,defer,sp", [
    (2, 1, 1, 2, False, False, False),   # dp2 x GA2 (no_sync micro-batch, then the sync pass)
    (2, 1, 1, 2, True, True, False),     # dp2 x GA2, ZeRO reduce-scatter, deferred grouped wgrad
    (4, 1, 2, 2, False, False, False),   # pp2 x dp2 1F1B with DDP buckets
    (4, 1, 2, 2, True, False, False),    # pp2 x dp2 + ZeRO (tied embedding shards must line up)
    (8, 2, 2, 2, True, True, True),      # the BASELINE layout tp2 pp2 dp2 + SP + ZeRO
])
def test_ddp_gradient_accumulation_matches_single_process(world, tp, pp, nmb, zero, defer, sp):
    """Reduced gradients after multi-micro-batch steps under DDP equal the full-batch gradients."""
    ref_loss, ref = W.gpt_reference()
    outs = run_workers(W.gpt_layout_worker, world, tp, pp, nmb, zero, defer, sp)
    for _, grads, meta in outs:
        _check_tp_grads(ref, grads, meta, tp)


@pytest.mark.parametrize("schedule", ["zb", "zbh2"])
@pytest.mark.parametrize("world,tp,pp,nmb,zero", [(4, 2, 2, 4, False), (8, 2, 2, 2, True)])
def test_w_fillers_in_exchange_waits_match_single_rank(schedule, world, tp, pp, nmb, zero):
    """SMDT_W_FILL: a pass's W GEMMs stay queued into the next forward and are issued one per
    TP-exchange wait (tensor_parallel.fill_exchange_wait), the rest flushed at its end; the split
    schedules still give the single-process losses and reduced gradients, and fillers ran."""
    over = {"num_layers": 2}
    ref_loss, ref = W.gpt_reference(cfg_over=over)
    outs = run_workers(W.gpt_layout_worker, world, tp, pp, nmb, zero, True, True, schedule, over, True,
                       timeout=600)
    fills = 0
    for _, grads, meta in outs:
        _check_tp_grads(ref, grads, meta, tp)
        fills += meta["wgrad_stats"].get("fills", 0)
    # zbh2 on pp2 with 2 micro-batches runs every forward ahead of every backward: nothing to fill
    assert (fills > 0) == (nmb > 2 or schedule == "zb"), fills
    for loss, _, meta in outs:
        if meta["pp_rank"] == pp - 1:
            per = 4 // (world // (tp * pp))
            want = ref_loss[meta["dp_rank"] * per:(meta["dp_rank"] + 1) * per]
            torch.testing.assert_close(loss.reshape(want.shape), want, atol=2e-4, rtol=2e-4)


@pytest.mark.parametrize("schedule", ["1f1b", "zb", "zbh1", "zbh2"])
@pytest.mark.parametrize("world,tp,pp,nmb,zero,sp,layers", [
    (4, 2, 2, 4, False, True, 2),      # tp2 pp2 + SP, 4 micro-batches of 1
    (4, 1, 4, 4, False, False, 4),     # pp4: three ranks with a cooldown, zbh1 holds up to 4 W
    (8, 2, 2, 2, True, True, 2),       # the BASELINE layout tp2 pp2 dp2 + SP + ZeRO
])
def test_split_backward_schedules_match_single_rank(schedule, world, tp, pp, nmb, zero, sp, layers):
    """The zero-bubble split backward (train/schedules.py: W GEMMs after the input gradient is
    sent; zbh1 also holds the last r + 1 passes' W of rank r until its final B; zbh2 runs
    2 (pp - r - 1) forwards ahead and holds the last 2 (r + 1) passes' W) gives the
    single-process losses and reduced gradients, with the deferred wgrad queue active on CPU."""
    over = {"num_layers": layers}
    ref_loss, ref = W.gpt_reference(cfg_over=over)
    outs = run_workers(W.gpt_layout_worker, world, tp, pp, nmb, zero, True, sp, schedule, over, timeout=600)
    for _, grads, meta in outs:
        _check_tp_grads(ref, grads, meta, tp)
        ws = meta["wgrad_stats"]
        assert ws["items"] > 0, ws                       # the weight gradients went through the queue
        # zbh1: rank r (>= 1) held its last r + 1 passes' W and merged them with the sync pass's
        # zbh2: every rank holds >= 2 passes' W (2 (r + 1) of them) and merges them
        held = (schedule == "zbh1" and meta["pp_rank"] >= 1) or schedule == "zbh2"
        assert (ws["max_segments"] >= 2) == held, (schedule, meta["pp_rank"], ws)
    for loss, _, meta in outs:
        if meta["pp_rank"] == pp - 1:
            per = 4 // (world // (tp * pp))
            want = ref_loss[meta["dp_rank"] * per:(meta["dp_rank"] + 1) * per]
            torch.testing.assert_close(loss.reshape(want.shape), want, atol=2e-4, rtol=2e-4)


@pytest.mark.parametrize("world", [2, 4])
def test_sp_linear_rings_overlap_wgrad_with_comm(world):
    """Collective-matmul SP linears: numerics match plain linears, and in backward each ring's last
    transfer is launched BEFORE the weight-gradient GEMM runs and waited for only AFTER it."""
    for ev in run_workers(W.tp_overlap_order_worker, world):
        bwd = ev[ev.index("backward") + 1:]
        # row linear backward (ring all-gather) first, then the column linear (ring reduce-scatter)
        steps = world - 1
        assert bwd.count("launch") == 2 * steps
        col = bwd[bwd.index("wgrad") + 1:]          # after the row linear's own wgrad
        i_w = col.index("wgrad")
        assert "launch" in col[:i_w], col             # column dgrad ring launched first
        assert col[i_w + 1:] and set(col[i_w + 1:]) == {"wait"}, col   # last transfer waited after the wgrad


def test_pipeline_output_deallocation_keeps_backward_exact():
    """deallocate_pipeline_outputs: a sent activation keeps only its graph (1-element data) and the
    engine-level backward still produces the exact input gradient."""
    from smdt_amd.train import schedules as S
    S.configure_p2p()
    x = torch.randn(8, 4, requires_grad=True)
    w = torch.randn(4, 4)
    out = torch.tanh(x @ w)
    g = torch.randn(8, 4)
    ref = torch.autograd.grad(torch.tanh(x @ w), x, g)[0]
    S._drop_output(out)
    assert out.numel() == 1
    S._run_backward(out, g)
    torch.testing.assert_close(x.grad, ref)


def test_ring_exchange_p2p_flag_is_rejected():
    import argparse
    from smdt_amd.train import schedules as S
    with pytest.raises(ValueError, match="ring_exchange"):
        S.configure_p2p(argparse.Namespace(use_ring_exchange_p2p=True))
    S.configure_p2p()


def test_distribute_saved_activations_shards_checkpoint_inputs():
    """--distribute-saved-activations: full-recompute gradients unchanged, and each TP rank keeps
    only a 1/tp slice of every checkpointed layer input (fewer saved bytes than plain recompute)."""
    ref_loss, ref = W.gpt_reference()
    full = {"recompute_granularity": "full", "recompute_method": "uniform"}
    plain = run_workers(W.saved_bytes_worker, 2, 2, full)
    dist_ = run_workers(W.saved_bytes_worker, 2, 2, {**full, "distribute_saved_activations": True})
    for loss, grads, meta, _ in dist_:
        _close(loss, ref_loss)
        _check_tp_grads(ref, grads, meta, 2)
    assert dist_[0][3] < plain[0][3], (dist_[0][3], plain[0][3])


def test_selective_recompute_drops_attention_scores():
    """Selective recompute (unfused attention): identical gradients, fewer bytes saved in forward
    (the [b, np, s, s] scores / probabilities are recomputed)."""
    outs = {g: run_workers(W.saved_bytes_worker, 1, 1, {"use_flash_attn": False, "recompute_granularity": g})[0]
            for g in (None, "selective")}
    for n, g in outs[None][1].items():
        torch.testing.assert_close(outs["selective"][1][n], g, atol=1e-6, rtol=1e-5)
    assert outs["selective"][3] < outs[None][3]


def test_rampup_batch_size_calculator():
    from smdt_amd.train.arguments import MicroBatchCalculator
    c = MicroBatchCalculator(global_batch_size=32, micro_batch_size=2, dp=2, rampup=[8, 8, 96])
    seen = []
    consumed = 0
    while consumed <= 140:
        seen.append(c.update(consumed))
        consumed += seen[-1]
    assert seen[0] == 8 and seen[-1] == 32 and seen == sorted(seen)
    assert set(seen) == {8, 16, 24, 32}                  # +8 every 96 / 3 = 32 samples
    assert c.num_micro_batches == 32 // 4
    with pytest.raises(ValueError):
        MicroBatchCalculator(32, 2, 2, rampup=[6, 8, 96])  # not a multiple of mbs x dp


def test_fused_norms_wait_for_their_parameter_gather():
    """The layers call ``Norm.fused`` instead of the norm's forward(), so nn.Module never runs its
    forward pre-hooks: the overlapped ZeRO parameter all-gather's wait (a pre-hook flagged
    ``_smdt_gather_wait``) must still run there, or the norm reads weights whose all-gather is in
    flight (the source of an intermittent ZeRO + overlap-param-gather mismatch on CPU)."""
    from smdt_amd.models.transformer import ParallelTransformerLayer, TransformerConfig
    cfg = TransformerConfig(num_layers=1, hidden_size=32, num_attention_heads=4, max_position_embeddings=16,
                            padded_vocab_size=64, hidden_dropout=0.0, attention_dropout=0.0, use_flash_attn=False)
    layer = ParallelTransformerLayer(cfg, 0)
    calls = []

    def wait(mod, inp):
        calls.append(mod)
    wait._smdt_gather_wait = True
    other = []
    layer.input_norm.register_forward_pre_hook(wait)
    layer.post_attention_norm.register_forward_pre_hook(wait)
    layer.post_attention_norm.register_forward_pre_hook(lambda m, i: other.append(m))   # unflagged: not run
    x = torch.randn(8, 2, 32, dtype=layer.input_norm.weight.dtype)
    layer(x, None, None)
    assert calls == [layer.input_norm, layer.post_attention_norm]
    assert other == []


def test_lm_head_ce_gate_and_cpu_loss_path():
    """The fused LM-head CE is a HIP-only path: on CPU tensors (and with TP > 1) the GPT loss goes
    through the separate linear + cross_entropy, whose per-token loss matches F.cross_entropy."""
    import torch.nn.functional as F
    from smdt_amd.ops import functional as SF
    from smdt_amd.parallel import tensor_parallel as tp
    torch.manual_seed(0)
    h = torch.randn(8, 2, 16, dtype=torch.bfloat16)
    w = torch.randn(64, 16, dtype=torch.bfloat16)
    assert not tp.lm_head_ce_ok(h, w, 1)
    assert not tp.lm_head_ce_ok(h, w, 2)
    tgt = torch.randint(0, 64, (8, 2))
    tgt[1, 1] = -100
    logits = (h.float() @ w.float().t())
    loss = SF.cross_entropy(logits, tgt)
    ref = F.cross_entropy(logits.view(-1, 64), tgt.view(-1), reduction="none", ignore_index=-100).view(8, 2)
    torch.testing.assert_close(loss, ref, atol=1e-5, rtol=1e-5)


@pytest.mark.parametrize("zero", [False, True])
def test_deterministic_reduce_is_rank_order_fold(zero):
    """SMDT_DETERMINISTIC_REDUCE / deterministic_reduce=True: the reduced gradient is exactly
    ((g_0 + g_1) + g_2 + g_3) / 4 over 4 ranks (values spanning 9 decades, so another association
    would differ in the last bits), whatever ring / tree the backend would have used."""
    import torch as _t
    outs = run_workers(W.deterministic_fold_worker, 4, zero)
    n = outs[0][0].numel()
    parts = []
    for r in range(4):
        g = _t.Generator().manual_seed(100 + r)
        parts.append(_t.randn(n, generator=g) * _t.logspace(-6, 3, n))
    want = ((parts[0] + parts[1]) + parts[2]) + parts[3]
    want = want / 4
    for got, ranges in outs:
        for s, e in ranges:
            assert _t.equal(got[s:e], want[s:e])


@pytest.mark.parametrize("tp,sp,pp", [(2, True, 1), (2, False, 1), (4, True, 1), (2, True, 2)])
def test_vocab_parallel_fused_lm_head_ce_matches_single_rank(tp, sp, pp, monkeypatch):
    """The vocab-parallel LM head + CE as one op (tensor_parallel.VocabParallelLMHeadCE: one pass
    over the logit slice, one all-gather of the [3, tokens] row statistics, the one-hot subtracted
    at one element per row, the row scale applied on the hidden side in the backward) on its CPU
    reference path: losses and every gradient equal single-rank training, with and without SP,
    at TP 4 and at the tp2 pp2 + SP layout of the N = 8 BASELINE point."""
    monkeypatch.setenv("SMDT_LM_HEAD_CE_CPU", "1")
    ref_loss, ref = W.gpt_reference()
    outs = run_workers(W.gpt_tp_worker, tp * pp, tp, pp, sp)
    for loss, grads, meta in outs:
        if pp == 1:
            _close(loss, ref_loss)
        _check_tp_grads(ref, grads, meta, tp)
    if pp > 1:
        last = [o for o in outs if o[2]["pp_rank"] == 1][0]
        torch.testing.assert_close(last[0].view(-1), ref_loss.view(-1), atol=2e-4, rtol=2e-4)


def test_vocab_parallel_fused_ce_path_is_taken(monkeypatch):
    """The gate: off for fp32 CPU tensors unless SMDT_LM_HEAD_CE_CPU=1, never at TP 1."""
    from smdt_amd.parallel import tensor_parallel as tp
    h = torch.zeros(4, 2, 16)
    w = torch.zeros(64, 16)
    assert not tp.vp_lm_head_ce_ok(h, w, 2)
    monkeypatch.setenv("SMDT_LM_HEAD_CE_CPU", "1")
    assert tp.vp_lm_head_ce_ok(h, w, 2) and not tp.vp_lm_head_ce_ok(h, w, 1)


def test_pending_add_ledger_unit():
    """A summand hung on a tensor must be taken before a check point (tensor_parallel ledger)."""
    from smdt_amd.parallel import tensor_parallel as tp
    t, x2 = torch.ones(4), torch.full((4,), 2.0)
    t = tp.set_pending_add(t, x2, "forward output")
    assert isinstance(t, tp.PendingPartial) and t.shape == (4,) and t.dtype == torch.float32
    assert tp.take_pending_add(t) is x2 and not hasattr(t, "_smdt_add")
    assert type(tp.plain(t)) is torch.Tensor and torch.equal(t, torch.ones(4))
    tp.check_pending_adds("after take")            # nothing pending: no error
    # the forward guard: any read of a pending output other than the fused norm's raises ...
    u = tp.set_pending_add(torch.ones(4), x2, "forward output")
    with pytest.raises(RuntimeError, match="another consumer"):
        u * 3
    # ... and without it (SMDT_DEFER_RS_GUARD=0) the ledger still catches the untaken summand
    prev = tp._GUARD
    tp._GUARD = False
    try:
        w = tp.set_pending_add(torch.ones(4), x2, "forward output")
        v = w * 3                                    # a consumer that is not the fused norm
        assert not hasattr(v, "_smdt_add")
        with pytest.raises(RuntimeError, match="never added"):
            tp.check_pending_adds("test")
        w = tp.set_pending_add(torch.ones(4), x2, "forward output")
        assert torch.equal(tp.materialize_add(w), torch.full((4,), 3.0))
        tp.check_pending_adds("after materialize")
    finally:
        tp._GUARD = prev
    u2 = tp.set_pending_add(torch.ones(4), x2, "forward output")
    m = tp.materialize_add(u2)
    assert type(m) is torch.Tensor and torch.equal(m, torch.full((4,), 3.0))
    tp.check_pending_adds("after guarded materialize")


def test_deferred_rs_add_with_a_forward_hook_materializes():
    """tp2 + SP (Gloo): a forward hook on a row-parallel linear of the layer stack turns the
    deferred reduce-scatter combine off, so the hook sees the complete output (equal to the run
    with SMDT_DEFER_RS_ADD=0) and the loss is unchanged. With the hook check disabled, the hook's
    read of the pending output raises (the forward guard, ``PendingPartial``); mutation arm: with
    that guard off too, the hook silently sees the output without the peer's partial."""
    base = run_workers(W.deferred_add_worker, 2, "hook", True, False)
    hooked = run_workers(W.deferred_add_worker, 2, "hook", True, True)
    caught = run_workers(W.deferred_add_worker, 2, "hook", False, True)
    unguarded = run_workers(W.deferred_add_worker, 2, "hook", False, True, False)
    for (l0, h0, _), (l1, h1, s1), (l2, _, s2), (_, h3, s3) in zip(base, hooked, caught, unguarded):
        assert isinstance(l1, torch.Tensor), l1
        _close(l1, l0)
        _close(h1, h0)
        assert s1["rs_add_to_norm"] == 0 and s2["rs_add_to_norm"] > 0 and s3["rs_add_to_norm"] > 0
        assert isinstance(l2, str) and "another consumer" in l2, l2
        assert (h3 - h0).abs().max() > 1e-3


def test_deferred_rs_add_second_consumer_raises():
    """tp2 + SP (Gloo) with the combine deferred: a model variant that reads the attention output
    (a pending row-parallel output) before handing it to the fused norm raises at that read (the
    forward guard) instead of computing with this rank's partial sum."""
    for out, _, _ in run_workers(W.deferred_add_worker, 2, "second_consumer"):
        assert isinstance(out, str) and "another consumer" in out, out


@pytest.mark.parametrize("case", ["plain_norm", "bwd"])
def test_deferred_rs_add_unconsumed_summand_raises(case):
    """tp2 + SP (Gloo) with the combine deferred, but the summand's consumer is not the fused norm:
    a model variant whose norm never takes it (forward), or a backward consumer of a deferred
    input-gradient summand that is not the fused norm kernel (the case of a norm output with a
    second consumer, whose summed gradient drops the attribute). It raises instead of returning a
    loss / gradients without the peer's partial: the forward guard at the plain norm's first read,
    the ledger for the backward (and for the forward with the guard off)."""
    for out, _, _ in run_workers(W.deferred_add_worker, 2, case):
        want = "another consumer" if case == "plain_norm" else "never added"
        assert isinstance(out, str) and want in out, out
    if case == "plain_norm":
        for out, _, _ in run_workers(W.deferred_add_worker, 2, case, True, True, False):
            assert isinstance(out, str) and "never added" in out, out


def test_link_standin_env_parsing(monkeypatch):
    """SMDT_LINK_STANDIN: ``relay`` / ``<GB/s>:<workgroups>`` select the paced ring stand-in,
    ``direct[:<GB/s per link>[:<workgroups>]]`` the paced direct-engine stand-in (TP4 / TP8 only:
    at tp 2 it warns and the exchanges stay in-line copies); unset / 0 / off: neither."""
    import warnings

    from smdt_amd.comm import loopback as lb
    from smdt_amd.parallel import state as ps
    cases = {"": (None, None), "0": (None, None), "off": (None, None), "relay": ((256.0, 64), None),
             "192:32": ((192.0, 32), None), "300": ((300.0, 64), None), "direct": (None, (64.0, 32)),
             "direct:80": (None, (80.0, 32)), "direct:80:16": (None, (80.0, 16))}
    for v, (ring, direct) in cases.items():
        monkeypatch.setenv("SMDT_LINK_STANDIN", v)
        assert lb.link_standin() == ring and lb.direct_standin() == direct, v
    monkeypatch.setenv("SMDT_LINK_STANDIN", "direct")
    ps.destroy_model_parallel()
    try:
        with warnings.catch_warnings(record=True) as w:
            warnings.simplefilter("always")
            st = ps.initialize_emulated_tensor_parallel(2)
        assert getattr(st, "tp_direct", None) is None
        assert any("TP4 / TP8 direct engine" in str(x.message) for x in w)
        ps.destroy_model_parallel()
        st = ps.initialize_emulated_tensor_parallel(4)
        td = st.tp_direct
        assert td is not None and td.world == 4 and td.rank == 0 and isinstance(td.eng, lb.PacedDirectEngine)
        assert (td.eng.gbps, td.eng.blocks) == (64.0, 32)
    finally:
        ps.destroy_model_parallel()


def test_switch_mlp_tensor_parallel_matches_single_rank():
    """``--num-experts`` under TP 2 (no SP): each expert is a tensor-parallel MLP, the router is
    replicated and routes identically on both ranks; loss and every (sharded) gradient equal the
    single-rank model's."""
    over = {"num_experts": 3}
    ref_loss, ref = W.gpt_reference(cfg_over=over)
    assert any(".experts.2." in n for n in ref)
    outs = run_workers(W.gpt_tp_worker, 2, 2, 1, False, over)
    for loss, grads, meta in outs:
        _close(loss, ref_loss)
        _check_tp_grads(ref, grads, meta, 2)
