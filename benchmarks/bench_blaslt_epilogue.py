"""Does hipBLASLt's fused bias+GELU epilogue run at the plain GEMM's speed on gfx950?

GPT-2 345M fc1 shape at the bench's tokens per step (65,536 x 1024 -> 4096, bf16):
torch.addmm (bias epilogue) + the separate bias/GELU kernel vs torch._addmm_activation
(hipBLASLt GELU_BIAS epilogue). Decides whether an epilogue-fused MLP path is worth wiring.
"""
import json
import torch


def timeit(fn, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(it):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / it


def main():
    M, K, N = 65536, 1024, 4096
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.03
    b = torch.randn(N, device="cuda", dtype=torch.bfloat16)
    res = {}
    res["mm_nobias"] = timeit(lambda: torch.mm(x, w.t()))
    res["addmm_bias"] = timeit(lambda: torch.addmm(b, x, w.t()))
    res["addmm_gelu_epilogue"] = timeit(lambda: torch._addmm_activation(b, x, w.t(), use_gelu=True))
    res["addmm_then_gelu"] = timeit(lambda: torch.nn.functional.gelu(torch.addmm(b, x, w.t()), approximate="tanh"))
    ref = torch.nn.functional.gelu(torch.addmm(b, x, w.t()).float(), approximate="tanh")
    got = torch._addmm_activation(b, x, w.t(), use_gelu=True).float()
    res["max_err_vs_tanh_gelu"] = (got - ref).abs().max().item()
    flop = 2 * M * K * N
    res.update({k + "_tflops": flop / v / 1e9 for k, v in list(res.items()) if k != "max_err_vs_tanh_gelu"})
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
