"""bench.py itself under torch.distributed.run with 2 / 4 / 8 gloo ranks on CPU (tiny shapes): the
paths the driver launches on an 8-GPU node start, run their layouts (DP + ZeRO-1 at N = 2 / 4, the
BASELINE tp2 pp2 dp2 + SP at N = 8, DP at N = 8), and rank 0 prints one well-formed JSON line whose
``phase_ms`` accounts for the measured step."""
import argparse
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

TINY = ["--num-layers", "4", "--hidden-size", "64", "--num-attention-heads", "4", "--seq-length", "32",
        "--vocab-size", "128", "--seqs-per-gpu", "4", "--steps", "2", "--warmup", "1"]


def _ns(**kw):
    base = dict(layout="baseline", tp=None, pp=None, sequence_parallel=None, seqs_per_gpu=32,
                micro_batch_size=None, grad_accum=None)
    base.update(kw)
    return argparse.Namespace(**base)


def test_choose_layout_per_world_size():
    import bench
    assert bench.choose_layout(_ns(), 1) == (1, 1, False, 32, 1)
    # N = 2 / 4: DP + ZeRO-1 (a tp2 pair shares one xGMI link: link-bound below N = 1, BENCHMARKS.md)
    assert bench.choose_layout(_ns(), 2) == (1, 1, False, 32, 1)
    assert bench.choose_layout(_ns(), 4) == (1, 1, False, 32, 1)
    assert bench.choose_layout(_ns(), 8) == (2, 2, True, 16, 8)      # BASELINE config #3
    assert bench.choose_layout(_ns(layout="dp"), 8) == (1, 1, False, 32, 1)
    assert bench.choose_layout(_ns(layout="tp"), 2) == (2, 1, True, 64, 1)
    assert bench.choose_layout(_ns(layout="tp"), 4) == (2, 2, True, 16, 8)
    tp, pp, sp, mbs, ga = bench.choose_layout(_ns(), 8)
    assert (pp - 1) / ga <= 0.2                                      # 1F1B bubble
    assert mbs * ga * 8 // (tp * pp) == 32 * 8                       # weak scaling: 32 seqs / GPU


def _run_bench(n, layout, tmp_path, extra=()):
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="1")
    from _dist import free_port
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", str(n), "--layout", layout] + TINY + list(extra)
    r = subprocess.run(cmd, cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


def _check_phases(rec):
    ph = rec["phase_ms"]
    parts = [v for k, v in ph.items() if k not in ("sum", "ms_per_step")]
    assert all(v >= 0 for v in parts), ph
    assert abs(sum(parts) - ph["sum"]) < 0.01 * max(1.0, ph["sum"])
    # the phases (CUDA events on GPU — recorded on two extra steps after the timed ones —, host
    # clocks on the timed steps of a CPU run) account for the whole measured step
    assert abs(ph["sum"] - rec["ms_per_step"]) <= 0.10 * rec["ms_per_step"], (ph, rec["ms_per_step"])


@pytest.mark.slow
@pytest.mark.parametrize("n,layout,want", [
    (2, "baseline", "tp1pp1dp2+zero1"),
    (4, "baseline", "tp1pp1dp4+zero1"),
    (8, "baseline", "tp2pp2dp2+sp+zero1"),
    (8, "dp", "tp1pp1dp8+zero1"),
])
def test_bench_ranks_gloo(n, layout, want, tmp_path):
    """The driver's N = 2 / 4 / 8 launches (gloo on CPU): one JSON line naming the layout, with a
    phase breakdown that sums to the step and per-axis collective accounting."""
    rec = _run_bench(n, layout, tmp_path)
    assert rec["n_gpus"] == n and rec["steps"] == 2 and rec["warmup"] == 1
    assert rec["config"]["parallelism"] == want and rec["config"]["layout"] == layout
    assert rec["config"]["global_batch"] == 4 * n
    assert rec["value"] > 0 and rec["final_loss"] > 0
    _check_phases(rec)
    comm = rec["comm"]
    assert "dp" in comm and comm["dp"]["MB"] > 0
    ops = comm["dp"]["ops"]
    assert any(k.startswith("reduce_scatter/") for k in ops) and any(k.startswith("all_gather/") for k in ops)
    assert rec["config"]["ddp_bucket"]["count"] >= 1
    if "tp2" in want:
        assert comm["tp"]["calls"] > 0 and comm["pp"]["calls"] > 0
        assert set(rec["phase_ms_by_pp_stage"]) == {"0", "1"}
        assert rec["config"]["pp_schedule"] == "zbh2"       # the N = 8 default schedule
        assert rec["phase_ms"]["tp_exchange_wait"] >= 0 and rec["phase_ms"]["pp_p2p_wait_and_bubble"] > 0


@pytest.mark.slow
@pytest.mark.parametrize("extra,want", [
    (["--pp-schedule", "1f1b"], "1f1b"),
    (["--pp-schedule", "zb"], "zb"),
    (["--pp-schedule", "zbh1"], "zbh1"),
    ([], "zbh2"),
    (["--vpp", "2"], "interleaved vpp2"),
])
def test_bench_pipeline_schedules_gloo(extra, want, tmp_path):
    """tp2 pp2 at N = 4 under each pipeline schedule bench.py can select (the zero-bubble split
    backward, zbh1, the default zbh2, and the interleaved virtual pipeline): the JSON names it."""
    rec = _run_bench(4, "tp", tmp_path, extra)
    assert rec["config"]["pp_schedule"] == want and rec["config"]["parallelism"] == "tp2pp2dp1+sp"
    assert rec["value"] > 0 and rec["final_loss"] > 0
    _check_phases(rec)


def test_bench_emulated_tp_rank(tmp_path):
    """--emulate-tp: one process times a TP rank's compute (sharded shapes, SP, ring-chunk GEMMs)
    with the collectives as local stand-ins (comm/loopback.py)."""
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", OMP_NUM_THREADS="1")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--emulate-tp", "2", "--micro-batch-size", "2",
           "--grad-accum", "2"] + TINY
    r = subprocess.run(cmd, cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    rec = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert rec["config"]["tp"] == 2 and "emulated" in rec["config"]["parallelism"]
    assert rec["metric"] == "emulated rank ms/step" and rec["unit"] == "ms" and not rec["higher_is_better"]
    assert rec["config"]["model"].endswith("vocab 256, seq 32)")   # padded to 128 x tp and rec["final_loss"] > 0


@pytest.mark.parametrize("stage", ["--emulate-first-stage", "--emulate-last-stage"])
def test_bench_emulated_pipeline_stage(tmp_path, stage):
    """The per-stage emulations predict_scaling.py times: the first stage without the LM head, the
    last without the embedding (its input a received activation), each with the F / B / W probe."""
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", OMP_NUM_THREADS="1")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--emulate-tp", "2", "--micro-batch-size", "2",
           "--grad-accum", "2", "--phase-probe", "2", stage] + TINY
    r = subprocess.run(cmd, cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    rec = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert set(rec["fbw_ms"]) >= {"F", "B", "W"}
    # an emulated rank is not a job throughput: its own metric, no headline fields
    assert rec["metric"] == "emulated rank ms/step" and rec["value"] == rec["ms_per_step"] > 0
    assert rec["vs_baseline"] is None and "model_tflops_per_gpu" not in rec


@pytest.mark.slow
def test_bench_n4_many_buckets_same_collective_order(tmp_path):
    """The round-3 one-GPU N = 4 rehearsal stalled in a bucket wait with ~75 buckets. The same
    many-bucket layout on CPU Gloo (buckets of 256 gradients: one per parameter tensor of the small model,
    as with the 16 MB buckets of the real one) completes, and the per-rank collective issue order
    (SMDT_COLLECTIVE_LOG) is identical on all four ranks."""
    env_extra = {"SMDT_COLLECTIVE_LOG": str(tmp_path / "clog")}
    old = {k: os.environ.get(k) for k in env_extra}
    os.environ.update(env_extra)
    try:
        rec = _run_bench(4, "baseline", tmp_path, ["--bucket-size", "256"])
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    assert rec["config"]["ddp_bucket"]["count"] >= 30, rec["config"]["ddp_bucket"]
    orders = []
    for r in range(4):
        lines = open(tmp_path / f"clog.rank{r}").read().splitlines()
        orders.append([ln.split(" ", 2)[2] for ln in lines])      # drop the index and timestamp
    assert len(orders[0]) > 2 * 30
    assert all(o == orders[0] for o in orders[1:])
