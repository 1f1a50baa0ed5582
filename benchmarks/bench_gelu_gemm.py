"""The GeLU-MLP GEMMs of the GPT-2 345M N = 1 step (fc1 forward with bias + GeLU, fc2 dgrad with the
GeLU backward), two ways, at the bench shape (mbs 64 x seq 1024 = 65,536 tokens, h 1024, ffn 4096):

  * ``gemm_tn``: the hand-written MFMA kernel with its epilogues (csrc/kernels/gemm_tn.hip, the
    default K5 path);
  (hipBLASLt's own GELU_AUX_BIAS / DGELU epilogues were measured at commit 69dd621 and removed:
    no gfx950 solution for GELU_AUX*, DGELU 3.5x slower and wrong; profiles/r6_gelu_neg/);
  * ``lib+ew``: the library GEMM (torch / hipBLASLt) and a separate elementwise pass.

Also checks each against an fp32 reference (tanh and erf GeLU) and prints one JSON line.

    python benchmarks/bench_gelu_gemm.py [--tokens 65536] [--reps 20]
"""
import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from smdt_amd.ops import _ext  # noqa: E402


def timed(fn, reps):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3   # us


def rel(a, b):
    return float((a.float() - b.float()).abs().max() / b.float().abs().max())


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--tokens", type=int, default=65536)
    p.add_argument("--hidden", type=int, default=1024)
    p.add_argument("--ffn", type=int, default=4096)
    p.add_argument("--reps", type=int, default=20)
    a = p.parse_args()
    C = _ext.ext()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    M, H, Fh = a.tokens, a.hidden, a.ffn
    bf = torch.bfloat16
    x = torch.randn(M, H, device=dev, dtype=bf)
    w1 = (torch.randn(Fh, H, device=dev) * H ** -0.5).to(bf)
    b1 = (torch.randn(Fh, device=dev) * 0.1).to(bf)
    w2 = (torch.randn(H, Fh, device=dev) * Fh ** -0.5).to(bf)
    dy = torch.randn(M, H, device=dev, dtype=bf)
    w2t = w2.t().contiguous()
    flops = 2.0 * M * H * Fh
    res = {"tokens": M, "gflop_per_gemm": round(flops / 1e9, 1)}

    # fp32 references (on a row slice: the full fp32 product would not change the verdict)
    R = 4096
    pre_ref = x[:R].float() @ w1.float().t() + b1.float()
    act_tanh = F.gelu(pre_ref, approximate="tanh")
    act_erf = F.gelu(pre_ref)
    g_ref = dy[:R].float() @ w2.float()
    pre_bf = pre_ref.to(bf).float()
    dz_tanh = torch.autograd.functional.vjp(lambda t: F.gelu(t, approximate="tanh"), pre_bf, g_ref)[1]
    dz_erf = torch.autograd.functional.vjp(lambda t: F.gelu(t), pre_bf, g_ref)[1]

    pre = torch.empty(M, Fh, device=dev, dtype=bf)
    act = torch.empty_like(pre)
    dz = torch.empty_like(pre)
    nob = torch.empty(0, device=dev, dtype=bf)
    # ---- gemm_tn
    fwd_tn = lambda: C.gemm_tn(x, w1, 2, b1, pre, act, 0, 0, None)  # noqa: E731
    fwd_tn()
    torch.cuda.synchronize()
    res["gemm_tn_fwd"] = {"us": round(timed(fwd_tn, a.reps), 1), "err_tanh": rel(act[:R], act_tanh),
                          "err_erf": rel(act[:R], act_erf),
                          "err_pre_nobias": rel(pre[:R], pre_ref - b1.float())}
    pre_keep = pre.clone()    # gemm_tn's pre-activation excludes the bias (its DGELU adds it back)
    bwd_tn = lambda: C.gemm_tn(dy, w2t, 3, b1, dz, None, 0, 0, pre_keep)  # noqa: E731
    bwd_tn()
    torch.cuda.synchronize()
    res["gemm_tn_dgelu"] = {"us": round(timed(bwd_tn, a.reps), 1), "err_tanh": rel(dz[:R], dz_tanh),
                            "err_erf": rel(dz[:R], dz_erf)}
    # ---- library GEMM + elementwise
    res["lib_fwd_gemm_us"] = round(timed(lambda: torch.matmul(x, w1.t(), out=pre), a.reps), 1)
    res["lib_dgrad_gemm_us"] = round(timed(lambda: torch.matmul(dy, w2, out=dz), a.reps), 1)
    res["ew_bias_gelu_us"] = round(timed(lambda: F.gelu(pre + b1, approximate="tanh"), a.reps), 1)
    for k, v in res.items():
        if isinstance(v, dict) and "us" in v:
            v["pflops"] = round(flops / v["us"] / 1e9, 3)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
