"""The QKV forward GEMM of the GPT-2 345M N = 1 step (65,536 tokens x 1024 -> 3072, with bias):
in the step trace it runs 467 us per call (0.88 PF/s) while TunableOp timed its tuned winner at 289
us. Times the candidate forms with the bench's TunableOp table loaded:

  * ``linear``: F.linear(x3d, w, b) (what ColumnParallelLinear calls);
  * ``addmm``: torch.addmm(b, x2d, w.t());
  * ``mm``: torch.mm(x2d, w.t()) without bias, and ``mm+bias``: then an in-place bias add;
  * ``gemm_tn``: the hand-written kernel with its bias epilogue.

Prints one JSON line (microseconds per call, median of --reps after warmup).

    python benchmarks/bench_qkv_bias.py [--tunableop 1]
"""
import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from smdt_amd.ops import _ext  # noqa: E402


def timed(fn, reps):
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    for s, e in evs:
        s.record()
        fn()
        e.record()
    torch.cuda.synchronize()
    ts = sorted(s.elapsed_time(e) * 1e3 for s, e in evs)
    return round(ts[len(ts) // 2], 1)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--tunableop", type=int, default=1)
    p.add_argument("--reps", type=int, default=25)
    p.add_argument("--seq", type=int, default=1024)
    p.add_argument("--mbs", type=int, default=64)
    a = p.parse_args()
    if a.tunableop:
        import torch.cuda.tunable as tun
        tun.enable(True)
        tun.tuning_enable(False)
        tun.set_filename("/tmp/smdt_qkv_unused.csv")
        tun.read_file(os.path.join(ROOT, "profiles", "tunableop", "gfx950_gpt345m_results.csv"))
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    bf = torch.bfloat16
    S, B, H = a.seq, a.mbs, 1024
    x = torch.randn(S, B, H, device=dev, dtype=bf)
    w = (torch.randn(3 * H, H, device=dev) * H ** -0.5).to(bf)
    b = (torch.randn(3 * H, device=dev) * 0.1).to(bf)
    x2 = x.view(-1, H)
    out = torch.empty(S * B, 3 * H, device=dev, dtype=bf)
    C = _ext.ext()
    res = {"M": S * B, "N": 3 * H, "K": H}
    res["linear"] = timed(lambda: F.linear(x, w, b), a.reps)
    res["addmm"] = timed(lambda: torch.addmm(b, x2, w.t()), a.reps)
    res["addmm_out"] = timed(lambda: torch.addmm(b, x2, w.t(), out=out), a.reps)
    res["mm"] = timed(lambda: torch.mm(x2, w.t()), a.reps)
    res["mm_out"] = timed(lambda: torch.mm(x2, w.t(), out=out), a.reps)
    res["mm+bias"] = timed(lambda: torch.mm(x2, w.t(), out=out).add_(b), a.reps)
    res["gemm_tn_bias"] = timed(lambda: C.gemm_tn(x2, w, 1, b, out, None, 0, 0, None), a.reps)
    ref = F.linear(x2.float(), w.float(), b.float())
    res["err_linear"] = float((F.linear(x, w, b).view(-1, 3 * H).float() - ref).abs().max())
    flops = 2.0 * S * B * H * 3 * H
    res["pflops"] = {k: round(flops / v / 1e9, 3) for k, v in res.items()
                     if k in ("linear", "addmm", "addmm_out", "mm", "mm_out", "mm+bias", "gemm_tn_bias")}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
