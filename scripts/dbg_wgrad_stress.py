"""Stress the grouped wgrad kernel: repeat one launch many times, count mismatching launches and
report where the bad elements sit (tile / wave / fragment coordinates) — a flaky-race hunt."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from smdt_amd.ops import _ext  # noqa: E402

C = _ext.ext()
torch.manual_seed(3)
shapes = [(2048, 1024, 1024), (2048, 384, 256), (1024, 3072, 1024), (4096, 256, 520)]
dys, xs, refs = [], [], []
for M, N, K in shapes:
    g = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    dys.append(g)
    xs.append(x)
    refs.append(g.float().t() @ x.float())
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
bad_launch = 0
for rep in range(reps):
    mgs = [torch.zeros(N, K, device="cuda") for (_, N, K) in shapes]
    C.wgrad_grouped(mgs, dys, xs)
    torch.cuda.synchronize()
    any_bad = False
    for pi, ((M, N, K), mg, ref) in enumerate(zip(shapes, mgs, refs)):
        bad = (mg - ref).abs() > 2e-2 * M ** 0.5 + 1e-3 * ref.abs()
        nb = int(bad.sum())
        if nb:
            any_bad = True
            idx = bad.nonzero()
            n, k = idx[0].tolist()
            d = (mg - ref)[n, k].item()
            print(f"rep {rep} prob {pi} bad {nb} first (n={n}, k={k}) tile ({n // 256},{k // 256}) "
                  f"local ({n % 256},{k % 256}) diff {d:.3f} ref {ref[n, k].item():.3f} "
                  f"rows {sorted(set(idx[:, 0].tolist()))[:8]} cols {sorted(set(idx[:, 1].tolist()))[:8]}", flush=True)
    bad_launch += any_bad
print(f"{os.environ.get('SMDT_WGRAD_MFMA')} split={os.environ.get('SMDT_WGRAD_TAIL_SPLIT')}: "
      f"{bad_launch}/{reps} launches wrong", flush=True)
