"""HBM rate of the fused Adam kernel on a flat GPT-2 345M-sized buffer (fp32 master / grad / m / v
+ bf16 model copy). SMDT_ADAM_U selects the form (0: grid-stride, 1 / 2 / 4 vectors per thread).

    python benchmarks/bench_adam.py [--n 354900000]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, ".")
from smdt_amd.ops import _ext  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=354_900_000)
    a = ap.parse_args()
    C = _ext.ext()
    dev = torch.device("cuda")
    n = a.n
    p = torch.randn(n, device=dev)
    g = torch.randn(n, device=dev) * 1e-3
    m = torch.zeros(n, device=dev)
    v = torch.zeros(n, device=dev)
    out = torch.empty(n, device=dev, dtype=torch.bfloat16)
    step = [0]

    def run():
        step[0] += 1
        C.adam(p, g, m, v, out, 1e-4, 0.9, 0.95, 1e-8, 0.01, step[0], True, None, None)
    for _ in range(3):
        run()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(10):
        run()
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / 10
    nbytes = n * (4 * 4 + 3 * 4 + 2)
    print(json.dumps({"SMDT_ADAM_U": os.environ.get("SMDT_ADAM_U", "default"), "n": n, "ms": round(ms, 4),
                      "TBps": round(nbytes / ms / 1e9, 2), "checksum": float(p[:1000].double().sum())}), flush=True)


if __name__ == "__main__":
    main()
