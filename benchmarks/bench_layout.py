"""TN vs NN for the forward linear GEMMs (hipBLASLt via torch, TunableOp table loaded as in bench.py):
y = x W^T as F.linear(x, W) (TN) against y = x Wt with Wt = W^T stored contiguous (NN), at M = 65536
(GPT-2 345M, micro-batch 64)."""
import json
import os

import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def timeit(fn, iters=20, warm=5):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ts = []
    for _ in range(iters):
        ev[0].record()
        fn()
        ev[1].record()
        torch.cuda.synchronize()
        ts.append(ev[0].elapsed_time(ev[1]))
    ts.sort()
    return ts[len(ts) // 2]


def main():
    import torch.cuda.tunable as tun
    tun.enable(True)
    tun.tuning_enable(False)
    tun.read_file(os.path.join(ROOT, "profiles", "tunableop", "gfx950_gpt345m_results.csv"))
    M = 65536
    for name, N, K in (("qkv", 3072, 1024), ("proj", 1024, 1024), ("fc1", 4096, 1024), ("fc2", 1024, 4096),
                       ("lm_head", 50304, 1024)):
        x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02
        wt = w.t().contiguous()
        t_tn = timeit(lambda: F.linear(x, w))
        t_nn = timeit(lambda: torch.matmul(x, wt))
        fl = 2.0 * M * N * K
        print(json.dumps({"gemm": name, "tn_ms": t_tn, "nn_ms": t_nn, "tn_tflops": fl / t_tn / 1e9,
                          "nn_tflops": fl / t_nn / 1e9}), flush=True)


if __name__ == "__main__":
    main()
