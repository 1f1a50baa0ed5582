"""bench.py itself under torch.distributed.run with 8 gloo ranks on CPU (tiny shapes): the 8-rank
path the driver launches on an 8-GPU node starts, runs the BASELINE layout (tp2 pp2 dp2 + SP) and
the DP layout, and rank 0 prints one well-formed JSON line."""
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
    assert bench.choose_layout(_ns(), 2) == (2, 1, True, 64, 1)
    assert bench.choose_layout(_ns(), 4) == (2, 2, True, 16, 8)
    assert bench.choose_layout(_ns(), 8) == (2, 2, True, 16, 8)      # BASELINE config #3
    assert bench.choose_layout(_ns(layout="dp"), 8) == (1, 1, False, 32, 1)
    tp, pp, sp, mbs, ga = bench.choose_layout(_ns(), 8)
    assert (pp - 1) / ga <= 0.2                                      # 1F1B bubble
    assert mbs * ga * 8 // (tp * pp) == 32 * 8                       # weak scaling: 32 seqs / GPU


@pytest.mark.slow
@pytest.mark.parametrize("layout,want", [("baseline", "tp2pp2dp2+sp+zero1"), ("dp", "tp1pp1dp8+zero1")])
def test_bench_eight_ranks_gloo(layout, want, tmp_path):
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="1")
    from _dist import free_port
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "8",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "8", "--layout", layout] + TINY
    r = subprocess.run(cmd, cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 8 and rec["steps"] == 2 and rec["warmup"] == 1
    assert rec["config"]["parallelism"] == want
    assert rec["config"]["global_batch"] == 4 * 8
    assert rec["value"] > 0 and rec["final_loss"] > 0
