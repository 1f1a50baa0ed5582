"""Per-collective accounting (comm/stats.py) and the auto-sized DP gradient buckets
(comm/buckets.py), on CPU / gloo."""
import os
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from _dist import run_workers  # noqa: E402

N8_RANK_PARAMS = 89_000_000   # GPT-2 345M at tp2 pp2: ~355 M / 4 parameters per rank


def test_bucket_size_rule():
    from smdt_amd.comm.buckets import MAX_BYTES, MIN_BYTES, NOMINAL_BYTES, choose_bucket_bytes
    grads = N8_RANK_PARAMS * 4
    assert choose_bucket_bytes(grads) == NOMINAL_BYTES
    assert grads // choose_bucket_bytes(grads) >= 4
    # 30 us launch latency at 100 GB/s: 10 % latency share at 27 MB
    assert choose_bucket_bytes(grads, 30e-6, 100e9) == int(9 * 30e-6 * 100e9)
    assert choose_bucket_bytes(grads, 1e-6, 100e9) == MIN_BYTES
    assert choose_bucket_bytes(grads, 1e-3, 100e9) == MAX_BYTES
    assert choose_bucket_bytes(40 << 20) == 10 << 20              # >= 4 buckets on small models
    assert choose_bucket_bytes(1 << 20) == 1 << 20                 # floor


def _ddp_buckets(rank, world, nparams):
    import torch.distributed as dist
    import torch.nn as nn
    from smdt_amd.comm import buckets
    from smdt_amd.parallel import state as ps
    from smdt_amd.parallel.distributed import DistributedDataParallel
    dist.init_process_group("gloo")
    ps.initialize_model_parallel(1, 1)
    width = 4096
    layers = max(1, nparams // (width * width))
    model = nn.Sequential(*[nn.Linear(width, width, bias=False) for _ in range(layers)])
    ddp = DistributedDataParallel(model, use_distributed_optimizer=True)
    out = (len(ddp.buckets), ddp.bucket_size, dict(buckets.TUNED), sum(p.numel() for p in model.parameters()))
    dist.destroy_process_group()
    return out


@pytest.mark.slow
def test_ddp_auto_buckets_at_n8_rank_size():
    """At the per-rank parameter count of the N = 8 layout the auto size gives >= 4 buckets, so the
    first reduce-scatter launches early in backward."""
    res = run_workers(_ddp_buckets, 2, N8_RANK_PARAMS, timeout=600)
    count, elems, tuned, numel = res[0]
    assert numel >= 0.9 * N8_RANK_PARAMS
    assert count >= 4 and res[1][0] == count
    assert 8 << 20 <= elems * 4 <= 32 << 20
    assert tuned["source"] == "nominal" and tuned["bucket_MB"] == elems * 4 / 2 ** 20


def _stats_worker(rank, world):
    import torch.distributed as dist
    from smdt_amd.comm import stats
    from smdt_amd.parallel import state as ps
    stats.enable(True, cuda=False)
    dist.init_process_group("gloo")
    ps.initialize_model_parallel(1, 1)
    st = ps.get_state()
    x = torch.ones(1 << 16)
    for _ in range(3):
        stats.begin_step()
        with stats.blocking("all_reduce", st.dp_group, x.numel() * 4):
            dist.all_reduce(x, group=st.dp_group)
        stats.mark("fwd_bwd")
        h = dist.reduce_scatter_tensor(torch.empty(x.numel() // world), x, group=st.dp_group, async_op=True)
        stats.collective("reduce_scatter", st.dp_group, x.numel() * 4, work=h)
        with stats.waiting("dp"):
            h.wait()
        stats.mark("grad_sync")
        stats.mark("optimizer")
        stats.end_step()
    out = stats.summary()
    stats.enable(False)
    dist.destroy_process_group()
    return out


def test_stats_accounting_gloo():
    res = run_workers(_stats_worker, 2)
    for out in res:
        assert out["steps"] == 3
        dp = out["comm"]["dp"]
        assert dp["calls"] == 2 and abs(dp["MB"] - 2 * (1 << 16) * 4 / 1e6) < 1e-3
        ar = dp["ops"]["all_reduce/gloo"]     # labelled by the group's library
        assert ar["ms"] > 0 and ar["busbw_GBps"] is not None and ar["ranks"] == 2
        ph = out["phase_ms"]
        # the blocking all-reduce sat inside forward/backward: it is a DP wait, not compute
        assert ph["other_comm_wait"] == 0 and ph["dp_param_gather_wait"] > 0
        assert abs(ph["sum"] - sum(v for k, v in ph.items() if k != "sum")) < 1e-2


def test_stats_off_is_inert():
    from smdt_amd.comm import stats
    stats.enable(False)
    stats.begin_step()
    with stats.waiting("tp"):
        pass
    stats.collective("all_reduce", None, 10)
    stats.end_step()
    assert not stats.active()


def test_xgmi_timeout_falls_back_to_rccl():
    """an injected engine timeout on ONE rank (step 2's first reduce-scatter)
    switches both ranks to the default transport at the same step, with one warning; the failed
    step is skipped, parameters are repaired, every loss stays finite and the replicas agree."""
    import dist_workers as W
    res = run_workers(W.xgmi_fallback_worker, 2, 0, 2)
    for r, out in enumerate(res):
        assert out["finite"], out
        assert out["replicas_equal"], out
        assert len(out["events"]) == 1 and out["events"][0]["error"] == 1
        # deactivated at the start of step 3, before its forward, on both ranks
        assert out["active"] == [True, True, False, False, False, False], out["active"]
    assert res[0]["active"] == res[1]["active"]
    assert res[0]["warned"] and not res[1]["warned"]
