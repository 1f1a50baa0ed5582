"""Hand-written TN GEMM (csrc/kernels/gemm_tn.hip) against torch's hipBLASLt / rocBLAS GEMM
(with the committed TunableOp winners, as bench.py runs it) at the GPT-2 345M step shapes
(64 x 1024 tokens): the forward linears F.linear(x, W) and the TN dgrads F.linear(dY, W^T).

Interleaved rounds in ONE process (cdna_hip_programming.md §5.4 rule 24), random operands
(rule 25). Also times the fc1 forward with its bias + GeLU epilogue against F.linear followed by
the standalone bias_act_fwd kernel (the unfused path of the training step).

    python benchmarks/bench_gemm_tn.py [--m 65536] [--rounds 5] [--reps 20]
"""
import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from smdt_amd.ops import _ext  # noqa: E402

TUNED = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles", "tunableop",
                     "gfx950_gpt345m_results.csv")

SHAPES = {  # name: (N, K) of out[M, N] = a[M, K] . b[N, K]^T
    "qkv_fwd": (3072, 1024),
    "proj_fwd": (1024, 1024),
    "fc1_fwd": (4096, 1024),
    "fc2_fwd": (1024, 4096),
    "qkv_dgrad": (1024, 3072),
    "fc1_dgrad": (1024, 4096),
    "fc2_dgrad": (4096, 1024),
    # tp2 stage-rank ring chunks (run with --m 16384)
    "fc1_chunk": (2048, 1024),
    "qkv_chunk": (1536, 1024),
}


def timeit(fn, reps):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--m", type=int, default=65536)
    p.add_argument("--rounds", type=int, default=5)
    p.add_argument("--reps", type=int, default=20)
    p.add_argument("--tunableop", type=int, default=1)
    p.add_argument("--only", nargs="*", default=None)
    p.add_argument("--max-blocks", type=int, default=0)
    p.add_argument("--ablate", nargs="*", type=int, default=None,
                   help="diagnostic kernel variants (VAR bits: 1 no DMA, 2 no fragment reads, "
                        "4 no stagger, 8 no stores) timed on the --only shapes instead of the A/B")
    a = p.parse_args()
    if a.tunableop and os.path.exists(TUNED):
        import tempfile
        import torch.cuda.tunable as tun
        tun.enable(True)
        tun.tuning_enable(False)
        tun.set_filename(os.path.join(tempfile.gettempdir(), "bench_gemm_tn_unused.csv"))
        tun.read_file(TUNED)
    C = _ext.ext()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    M = a.m
    res = {}
    names = a.only or list(SHAPES)
    data = {}
    for n in names:
        N, K = SHAPES[n]
        x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
        w = torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        ref = F.linear(x, w)
        got = C.gemm_tn(x, w, 0, None, out, None, a.max_blocks)[0]
        err = ((got.float() - ref.float()).abs().max() / ref.float().abs().max()).item()
        data[n] = (x, w, out)
        res[n] = {"N": N, "K": K, "max_rel_err_vs_blaslt": err, "ours_ms": [], "lib_ms": []}
    if "fc1_fwd" in names:
        N, K = SHAPES["fc1_fwd"]
        x, w, out = data["fc1_fwd"]
        b = torch.randn(N, device=dev, dtype=torch.bfloat16) * 0.1
        o2 = torch.empty_like(out)
        pre, act = C.gemm_tn(x, w, 2, b, out, o2, a.max_blocks)
        h = F.linear(x, w)
        ract = C.bias_act_fwd(h, b, 0)
        eact = ((act.float() - ract.float()).abs().max()).item()
        res["fc1_bias_gelu"] = {"N": N, "K": K, "max_abs_err_vs_unfused": eact, "ours_ms": [], "lib_ms": []}
    if "fc2_dgrad" in names:
        # fc2 dgrad with the GeLU backward in the epilogue vs the library GEMM + bias_act_bwd
        N, K = SHAPES["fc2_dgrad"]
        dy, w2t, dout = data["fc2_dgrad"]
        b1 = torch.randn(N, device=dev, dtype=torch.bfloat16) * 0.1
        pre1 = torch.randn(M, N, device=dev, dtype=torch.bfloat16)
        got = C.gemm_tn(dy, w2t, 3, b1, dout, None, a.max_blocks, 0, pre1)[0].clone()
        ref = C.bias_act_bwd(torch.mm(dy, w2t.t()), pre1, b1, 0, False, None)[0]
        ed = ((got.float() - ref.float()).abs().max() / ref.float().abs().max()).item()
        res["fc2_dgrad_dgelu"] = {"N": N, "K": K, "max_rel_err_vs_unfused": ed, "ours_ms": [], "lib_ms": []}
    if a.ablate:
        out_ab = {}
        for n in names:
            x, w, out = data[n]
            N, K = SHAPES[n]
            fl = 2.0 * M * N * K
            ref = F.linear(x, w).float()
            for v in [0] + list(a.ablate):
                if not (v & 9) or v in (64, 1024):   # variants that compute the product: check it
                    got = C.gemm_tn(x, w, 0, None, out, None, a.max_blocks, v)[0].float()
                    err = ((got - ref).abs().max() / ref.abs().max()).item()
                    assert err < 1e-2, (n, v, err)
                ts = [timeit(lambda: C.gemm_tn(x, w, 0, None, out, None, a.max_blocks, v), a.reps)
                      for _ in range(a.rounds)]
                t = sorted(ts)[len(ts) // 2]
                out_ab[f"{n}/var{v}"] = round(t, 4)
                print(f"{n:12s} var {v:2d}: {t:.4f} ms ({fl / t / 1e9:.0f} TF/s)", flush=True)
                if n in ("fc1_fwd", "fc1_chunk") and v in (0, 64, 1024):   # bias + GeLU epilogue
                    bb = torch.randn(N, device=dev, dtype=torch.bfloat16) * 0.1
                    o2 = torch.empty_like(out)
                    ts = [timeit(lambda: C.gemm_tn(x, w, 2, bb, out, o2, a.max_blocks, v), a.reps)
                          for _ in range(a.rounds)]
                    t = sorted(ts)[len(ts) // 2]
                    out_ab[f"{n}/gelu/var{v}"] = round(t, 4)
                    print(f"{n:12s} gelu var {v:2d}: {t:.4f} ms ({fl / t / 1e9:.0f} TF/s)", flush=True)
        print(json.dumps({"M": M, "ablate_ms": out_ab}))
        return
    for r in range(a.rounds):
        for n in names:
            x, w, out = data[n]
            res[n]["ours_ms"].append(timeit(lambda: C.gemm_tn(x, w, 0, None, out, None, a.max_blocks), a.reps))
            res[n]["lib_ms"].append(timeit(lambda: torch.mm(x, w.t(), out=out), a.reps))
        if "fc1_fwd" in names:
            x, w, out = data["fc1_fwd"]
            res["fc1_bias_gelu"]["ours_ms"].append(
                timeit(lambda: C.gemm_tn(x, w, 2, b, out, o2, a.max_blocks), a.reps))
            res["fc1_bias_gelu"]["lib_ms"].append(
                timeit(lambda: C.bias_act_fwd(torch.mm(x, w.t(), out=out), b, 0), a.reps))
        if "fc2_dgrad" in names:
            res["fc2_dgrad_dgelu"]["ours_ms"].append(
                timeit(lambda: C.gemm_tn(dy, w2t, 3, b1, dout, None, a.max_blocks, 0, pre1), a.reps))
            res["fc2_dgrad_dgelu"]["lib_ms"].append(
                timeit(lambda: C.bias_act_bwd(torch.mm(dy, w2t.t(), out=dout), pre1, b1, 0, False, None), a.reps))
    tot_o = tot_l = 0.0
    for n, r in res.items():
        o = sorted(r["ours_ms"])[len(r["ours_ms"]) // 2]
        lb = sorted(r["lib_ms"])[len(r["lib_ms"]) // 2]
        fl = 2.0 * M * r["N"] * r["K"]
        r.update(ours_med_ms=round(o, 4), lib_med_ms=round(lb, 4), ours_tflops=round(fl / o / 1e9, 1),
                 lib_tflops=round(fl / lb / 1e9, 1), speedup=round(lb / o, 3))
        if n not in ("fc1_bias_gelu", "fc2_dgrad_dgelu"):
            tot_o += o
            tot_l += lb
        print(f"{n:14s} N {r['N']:5d} K {r['K']:5d}  ours {o:.4f} ms ({r['ours_tflops']:.0f} TF/s)  "
              f"lib {lb:.4f} ms ({r['lib_tflops']:.0f} TF/s)  x{r['speedup']:.3f}", flush=True)
    print(json.dumps({"M": M, "sum_ours_ms": round(tot_o, 4), "sum_lib_ms": round(tot_l, 4),
                      "shapes": {k: {kk: vv for kk, vv in v.items() if not kk.endswith("_ms") or "med" in kk}
                                 for k, v in res.items()}}))


if __name__ == "__main__":
    main()
