"""Which hipBLASLt GeLU epilogues have gfx950 bf16 solutions at the fc1 / fc2-dgrad shapes
(diagnostics for csrc/blaslt.cpp gemm_gelu). Prints one line per configuration: heuristic
candidate count (negative: error status)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from smdt_amd.ops import _ext  # noqa: E402

C = _ext.ext()
M, N, K = 65536, 4096, 1024
EPI = {"DEFAULT": 1, "BIAS": 4, "GELU": 32, "GELU_BIAS": 36, "GELU_AUX": 160, "GELU_AUX_BIAS": 164, "DGELU": 192,
       "DGELU_BGRAD": 208}
for name, e in EPI.items():
    for aux in (0, 1, 2):
        if e < 128 and aux:
            continue
        for bias in ((False, True) if e in (4, 36, 164, 208) else (False,)):
            for ta in (1, 0):
                for d in (1, 2):
                    n = C.gelu_probe(M, N, K, e, aux, bias, ta, d)
                    print(f"{name:14s} aux={aux} bias={int(bias)} transA={ta} D={'f32' if d == 2 else 'bf16'}: {n}",
                          flush=True)
