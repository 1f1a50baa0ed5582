"""Does the Infinity Cache (256 MB MALL) pay for chunking fc1 -> bias-GeLU -> fc2?

Times, at the GPT-2 345M MLP shape (M = 65536 tokens, h = 1024, ffn = 4096, bf16), the forward
chain fc1 GEMM -> bias-GeLU kernel -> fc2 GEMM run once over all M rows against the same chain run
over M / c row chunks back to back (each chunk's GEMM output re-read by the next kernel while it
may still sit in the MALL). Prints one JSON line per chunk count with per-kernel totals."""
import json
import os
import sys

import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch.cuda.tunable as tun
    tun.enable(True)
    tun.tuning_enable(False)
    tun.read_file(os.path.join(ROOT, "profiles", "tunableop", "gfx950_gpt345m_results.csv"))
    from smdt_amd.ops import functional as SF
    M, H, FF = 65536, 1024, 4096
    dev = "cuda"
    x = torch.randn(M, H, device=dev, dtype=torch.bfloat16)
    w1 = torch.randn(FF, H, device=dev, dtype=torch.bfloat16) * 0.02
    b1 = torch.randn(FF, device=dev, dtype=torch.bfloat16) * 0.02
    w2 = torch.randn(H, FF, device=dev, dtype=torch.bfloat16) * 0.02
    pre = torch.empty(M, FF, device=dev, dtype=torch.bfloat16)
    y = torch.empty(M, H, device=dev, dtype=torch.bfloat16)
    flush = torch.empty(512 << 20, device=dev, dtype=torch.uint8)

    def run(c, split_times):
        n = M // c
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(4 * c)]
        acts = []
        for i in range(c):
            xs = x[i * n:(i + 1) * n]
            ev[4 * i].record()
            torch.mm(xs, w1.t(), out=pre[i * n:(i + 1) * n])
            ev[4 * i + 1].record()
            a = SF.bias_gelu(pre[i * n:(i + 1) * n], b1, "tanh")
            ev[4 * i + 2].record()
            torch.mm(a, w2.t(), out=y[i * n:(i + 1) * n])
            ev[4 * i + 3].record()
            acts.append(a)
        torch.cuda.synchronize()
        for i in range(c):
            split_times[0] += ev[4 * i].elapsed_time(ev[4 * i + 1])
            split_times[1] += ev[4 * i + 1].elapsed_time(ev[4 * i + 2])
            split_times[2] += ev[4 * i + 2].elapsed_time(ev[4 * i + 3])
        return acts

    for c in (1, 2, 4, 8, 16):
        for _ in range(3):
            run(c, [0.0, 0.0, 0.0])
        t = [0.0, 0.0, 0.0]
        it = 10
        for _ in range(it):
            flush.zero_()
            run(c, t)
        t = [v / it for v in t]
        print(json.dumps({"chunks": c, "fc1_ms": round(t[0], 4), "bias_gelu_ms": round(t[1], 4),
                          "fc2_ms": round(t[2], 4), "total_ms": round(sum(t), 4)}), flush=True)


if __name__ == "__main__":
    main()
