#!/usr/bin/env python3
"""Per-rank compute of the N = 8 tp2 pp2 dp2 layout at different micro-batch sizes (one MI355X):
the balanced 13 | 11 stage shapes of benchmarks/predict_scaling.py with 256 sequences per replica
cut into micro-batches of 16 / 32 / 64."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "benchmarks"))
from predict_scaling import _TP2  # noqa: E402

out = {}
os.makedirs(os.path.join(ROOT, "gpurun_out", "predict_mbs"), exist_ok=True)
for mbs in (16, 32, 64):
    ga = 256 // mbs
    for name, extra in (("stage0", ["--num-layers", "13", "--emulate-first-stage"]), ("stage1", ["--num-layers", "11"])):
        cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "5", "--warmup", "2"] + extra + _TP2 + \
              ["--seqs-per-gpu", "256", "--micro-batch-size", str(mbs), "--grad-accum", str(ga)]
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=ROOT)
        with open(os.path.join(ROOT, "gpurun_out", "predict_mbs", f"{name}_mbs{mbs}.log"), "w") as f:
            f.write(r.stdout + r.stderr)
        if r.returncode:
            raise SystemExit(r.stderr[-2000:])
        rec = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
        out[f"{name}_mbs{mbs}"] = rec["ms_per_step"]
        print(f"{name} mbs {mbs} x {ga}: {rec['ms_per_step']:.1f} ms", flush=True)
for mbs in (16, 32, 64):
    t = max(out[f"stage0_mbs{mbs}"], out[f"stage1_mbs{mbs}"])
    m = 256 // mbs
    print(f"mbs {mbs}: per-rank {t:.1f} ms, 1F1B bubble {t / m:.1f} ms, interleaved vpp2 bubble {t / m / 2:.1f} ms")
