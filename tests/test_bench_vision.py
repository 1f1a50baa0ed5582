"""benchmarks/bench_vision.py (BASELINE config #2, Oxford-Pet DDP) under torch.distributed.run
with 2 and 8 Gloo ranks on CPU (tiny images): the multi-rank path starts, every rank trains with
the framework's bucketed DDP reducer, and rank 0 prints one JSON line naming the layout and the
gradient bucket size it ran with."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _run(n, model, tmp_path, extra=()):
    from _dist import free_port
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()),
           os.path.join(ROOT, "benchmarks", "bench_vision.py"), "--model", model, "--size", "32",
           "--batch", "2", "--dtype", "fp32", "--steps", "2", "--warmup", "1"] + list(extra)
    r = subprocess.run(cmd, cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


@pytest.mark.parametrize("n,bucket_mb", [(2, 8.0), (8, 0.0)])
def test_bench_vision_gloo_ranks(n, bucket_mb, tmp_path):
    rec = _run(n, "resnet50", tmp_path, ["--bucket-mb", str(bucket_mb)])
    assert rec["n_gpus"] == n and rec["value"] > 0
    cfg = rec["config"]
    assert cfg["parallelism"] == f"dp{n}" and cfg["backend"] == "gloo"
    b = cfg["ddp_bucket"]
    if bucket_mb:
        assert b["elements"] == int(bucket_mb * 2 ** 20 / 4) and b["MB"] == bucket_mb
        assert b["count"] >= 3, b      # ResNet-50's 25.6 M fp32 gradients over 8 MB buckets
    else:
        assert b["count"] >= 1 and b["MB"] > 0, b   # auto size (comm/buckets.py) is reported
    assert abs(rec["final_loss"]) < 100
