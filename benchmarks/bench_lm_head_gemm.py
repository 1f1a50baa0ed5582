"""The GPT-2 345M LM-head GEMMs as the N = 1 step issues them, with the committed TunableOp
table preloaded exactly as bench.py loads it: forward logits = F.linear(h, W) [65536 x 50304 x
1024] and the TN dgrad F.linear(D, W^T) [65536 x 1024 x 50304]; also the NN dgrad D @ W. Prints
per-call times; run under rocprofv3 --kernel-trace to see which library kernel each one takes.

    python benchmarks/bench_lm_head_gemm.py [--tunableop 1] [--reps 5]
"""
import argparse
import os
import sys
import tempfile

import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TUNED = os.path.join(ROOT, "profiles", "tunableop", "gfx950_gpt345m_results.csv")


def timeit(fn, reps):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--tunableop", type=int, default=1)
    p.add_argument("--reps", type=int, default=5)
    p.add_argument("--m", type=int, default=65536)
    a = p.parse_args()
    if a.tunableop:
        import torch.cuda.tunable as tun
        tun.enable(True)
        tun.tuning_enable(False)
        tun.set_filename(os.path.join(tempfile.gettempdir(), "lm_head_unused.csv"))
        tun.read_file(TUNED)
    dev = torch.device("cuda", 0)
    V, H, M = 50304, 1024, a.m
    h = torch.randn(M, H, device=dev, dtype=torch.bfloat16)
    w = torch.randn(V, H, device=dev, dtype=torch.bfloat16) * 0.02
    wt = w.t().contiguous()
    d = torch.randn(M, V, device=dev, dtype=torch.bfloat16) * 0.01
    fl = 2.0 * M * V * H
    for name, fn in (("fwd F.linear(h, W)", lambda: F.linear(h, w)),
                     ("dgrad TN F.linear(D, W^T)", lambda: F.linear(d, wt)),
                     ("dgrad NN D @ W", lambda: torch.mm(d, w))):
        t = timeit(fn, a.reps)
        print(f"{name:28s} {t:.3f} ms  {fl / t / 1e9:.0f} TF/s", flush=True)


if __name__ == "__main__":
    main()
