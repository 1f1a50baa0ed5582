"""One grouped wgrad launch in a FRESH process, exactly as tests/test_parallel_gpu.py builds it
(random base accumulators), reporting mismatches. argv[1]: 'clone' (test form) or 'zeros'."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from smdt_amd.ops import _ext  # noqa: E402

mode = sys.argv[1] if len(sys.argv) > 1 else "clone"
torch.manual_seed(3)
shapes = [(2048, 1024, 1024), (2048, 384, 256), (1024, 3072, 1024), (4096, 256, 520)]
mgs, dys, xs, refs = [], [], [], []
for M, N, K in shapes:
    g = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    base = torch.randn(N, K, device="cuda", dtype=torch.float32) if mode != "zeros" else torch.zeros(N, K, device="cuda")
    mgs.append(base.clone())
    dys.append(g)
    xs.append(x)
    refs.append(base + g.float().t() @ x.float())
if mode == "sync":
    torch.cuda.synchronize()
_ext.ext().wgrad_grouped(mgs, dys, xs)
torch.cuda.synchronize()
tot = 0
for pi, ((M, N, K), mg, ref) in enumerate(zip(shapes, mgs, refs)):
    bad = (mg - ref).abs() > 2e-2 * M ** 0.5 + 1e-3 * ref.abs()
    nb = int(bad.sum())
    tot += nb
    if nb:
        idx = bad.nonzero()
        n, k = idx[0].tolist()
        again = (mg - ref)[n, k].item()
        print(f"  prob {pi} bad {nb} first (n={n},k={k}) tile ({n // 256},{k // 256}) local ({n % 256},{k % 256}) "
              f"diff {again:.3f} rows {sorted(set(idx[:, 0].tolist()))[:6]} cols {sorted(set(idx[:, 1].tolist()))[:6]}")
print(f"{mode} {os.environ.get('SMDT_WGRAD_MFMA')} split={os.environ.get('SMDT_WGRAD_TAIL_SPLIT')}: bad={tot}")
