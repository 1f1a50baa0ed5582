"""TunableOp winners for the GEMM shapes of bench.py's multi-GPU layouts, tuned on ONE MI355X.

TunableOp keys its table by (op, layout, M, N, K, leading dims), so the shapes a TP=2 rank runs
can be tuned without the other rank: this script issues exactly the torch calls the
sequence-parallel ring collective-matmuls make (parallel/tensor_parallel.py: ``_mm_into`` /
``F.linear`` per chunk in forward, ``matmul`` per chunk in backward) and the vocab-parallel LM
head, for

    N = 1     tp1, micro-batch 64  (backward dgrad shapes)
    N = 2     tp2, micro-batch 64  (chunk rows = s / 2 * 64)
    N = 8     tp2, micro-batch 32  (chunk rows = s / 2 * 32; bench.py's N = 8 split since round 3)
    (micro-batch 16: the round-2 N = 4 / 8 splits)

GPT-2 345M: h = 1024, ffn 4096, 16 heads, vocab 50304 (padded for tp2: 25152 per rank).
Results go to ``--out`` (merge into profiles/tunableop/ with ``--merge``).

    python scripts/tune_gemm_shapes.py --out gpurun_out/tune/tp2.csv            # on the GPU
    python scripts/tune_gemm_shapes.py --out gpurun_out/tune/tp2.csv --merge-only  # then, here
"""
from __future__ import annotations

import argparse
import os

# one warmup call per candidate solution (the search covers every hipBLASLt / rocBLAS solution)
os.environ.setdefault("PYTORCH_TUNABLEOP_MAX_WARMUP_ITERATIONS", "1")
os.environ.setdefault("PYTORCH_TUNABLEOP_MAX_WARMUP_DURATION_MS", "1")

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

H, FFN, S = 1024, 4096, 1024
VOCAB_TP2 = 50304 // 2


def shapes(mbs_list=(64, 32, 16), n1=True):
    # Dgrad GEMMs run in the TN layout: dX = F.linear(dY, W^T) / torch.mm(dY, W^T.t(), out=)
    # with a contiguous W^T (parallel/tensor_parallel.py ``dgrad`` / ``dgrad_into``), so the
    # backward shapes below are "linear" / "mm" calls with N = in-features, K = out-features.
    # N = 1 (tp1, micro-batch 64): the backward dgrad GEMMs (the forward ones are tuned by
    # ``bench.py --tunableop 2``, whose first warmup step reaches them first)
    mt = S * 64
    out = [] if not n1 else [("linear", mt, H, 50304), ("linear", mt, H, FFN), ("linear", mt, FFN, H), ("linear", mt, H, H),
           ("linear", mt, H, 3 * H)]
    if n1 and os.environ.get("SMDT_TUNE_N1_FORWARD", "0") == "1":
        # N = 1 forward: qkv with bias (addmm), proj / fc1 / fc2 without (the bias goes to the
        # fused LN / bias-GeLU kernels), LM head
        out += [("addmm", mt, 3 * H, H), ("mm", mt, H, H), ("mm", mt, FFN, H), ("mm", mt, H, FFN),
                ("mm", mt, 50304, H)]
    for mbs in mbs_list:
        m = S // 2 * mbs  # one ring chunk of a sequence-parallel [s / tp, b, h] activation
        # forward column-parallel (qkv with bias, fc1 without: bias-GeLU is a separate kernel)
        out += [("addmm", m, 3 * H // 2, H), ("mm", m, FFN // 2, H)]
        # forward row-parallel chunks (proj, fc2)
        out += [("linear", m, H, H // 2), ("linear", m, H, FFN // 2)]
        # backward: column dgrad chunks F.linear(g[m, out/2], W^T[h, out/2]);
        # row dgrad chunks mm(g[m, h], W^T[in/2, h].t(), out=)
        out += [("linear", m, H, 3 * H // 2), ("linear", m, H, FFN // 2),
                ("mm", m, H // 2, H), ("mm", m, FFN // 2, H)]
        # vocab-parallel LM head, one ring chunk: forward mm into the gathered output, dgrad
        out += [("mm", m, VOCAB_TP2, H), ("linear", m, H, VOCAB_TP2)]
    return out


def run(kind, m, n, k, dev):
    a = torch.randn(m, k, device=dev, dtype=torch.bfloat16)
    if kind == "matmul":      # a[m, k] @ w[k, n]   (backward dgrad: NN)
        w = torch.randn(k, n, device=dev, dtype=torch.bfloat16)
        out = torch.empty(m, n, device=dev, dtype=torch.bfloat16)
        torch.matmul(a, w, out=out)
        a.matmul(w)
    else:                     # a[m, k] @ w[n, k]^T (forward: TN)
        w = torch.randn(n, k, device=dev, dtype=torch.bfloat16)
        out = torch.empty(m, n, device=dev, dtype=torch.bfloat16)
        if kind == "addmm":
            b = torch.randn(n, device=dev, dtype=torch.bfloat16)
            torch.addmm(b, a, w.t(), out=out)
        elif kind == "mm":
            torch.mm(a, w.t(), out=out)
        else:
            F.linear(a, w)
    torch.cuda.synchronize()


def merge(new_csv, table):
    keep = {}
    order = []
    for path in (table, new_csv):
        if not os.path.exists(path):
            continue
        for line in open(path):
            line = line.rstrip("\n")
            if not line:
                continue
            parts = line.split(",")
            key = (parts[0], parts[1]) if parts[0] != "Validator" else ("Validator", parts[1])
            if key not in keep:
                order.append(key)
            if path == table or parts[0] != "Validator":
                keep[key] = line
    with open(table, "w") as f:
        f.write("\n".join(keep[k] for k in order) + "\n")


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--out", default="gpurun_out/tune/tp2.csv")
    p.add_argument("--tune-ms", type=int, default=60)
    p.add_argument("--iters", type=int, default=5, help="timed iterations per candidate solution")
    p.add_argument("--skip-lm-head", type=int, default=1, help="skip the vocab GEMMs (~5 min of search each)")
    p.add_argument("--mbs", type=str, default="64,32,16", help="tp2 micro-batch sizes to tune")
    p.add_argument("--skip-n1", action="store_true", help="skip the N = 1 dgrad shapes")
    p.add_argument("--merge", action="store_true", help="merge --out into the committed table afterwards")
    p.add_argument("--merge-only", action="store_true", help="only merge an existing --out (no GPU)")
    a = p.parse_args()
    table = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles", "tunableop",
                         "gfx950_gpt345m_results.csv")
    if a.merge_only:
        merge(a.out, table)
        print(f"merged into {table}")
        return
    import torch.cuda.tunable as tun
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    tun.enable(True)
    tun.tuning_enable(True)
    tun.set_max_tuning_duration(a.tune_ms)
    tun.set_max_tuning_iterations(a.iters)
    tun.set_filename(a.out)
    dev = torch.device("cuda")
    import threading
    import time
    t_start = time.time()

    def beat():  # progress line every 30 s: one shape's search over every solution takes minutes
        while True:
            time.sleep(30)
            print(f"... tuning ({time.time() - t_start:.0f} s)", flush=True)
    threading.Thread(target=beat, daemon=True).start()
    for kind, m, n, k in shapes(tuple(int(x) for x in a.mbs.split(",")), not a.skip_n1):
        if a.skip_lm_head and max(n, k) > 8192:
            continue
        t0 = time.time()
        run(kind, m, n, k, dev)
        print(f"tuned {kind} M={m} N={n} K={k} in {time.time() - t0:.1f} s", flush=True)
    if a.merge:
        merge(a.out, table)
        print(f"merged into {table}")


if __name__ == "__main__":
    main()
