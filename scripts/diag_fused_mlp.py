"""Check the hipBLASLt epilogue-fused MLP on the GPT-2 345M shapes and time it against the unfused path."""
import sys
import torch
sys.path.insert(0, ".")
from smdt_amd.ops import _ext  # noqa: E402

C = _ext.ext()
M, H, F = 16384, 1024, 4096
x = torch.randn(M, H, device="cuda", dtype=torch.bfloat16)
w1 = torch.randn(F, H, device="cuda", dtype=torch.bfloat16) * 0.02
b1 = torch.randn(F, device="cuda", dtype=torch.bfloat16) * 0.1
w2 = torch.randn(H, F, device="cuda", dtype=torch.bfloat16) * 0.02
act = torch.empty(M, F, device="cuda", dtype=torch.bfloat16)
aux = torch.empty_like(act)
print("linear_gelu_fwd", C.linear_gelu_fwd(x, w1, b1, act, aux), flush=True)
dy = torch.randn(M, H, device="cuda", dtype=torch.bfloat16)
dpre = torch.empty_like(act)
bg = torch.empty(F, device="cuda", dtype=torch.float32)
print("linear_dgelu_bwd", C.linear_dgelu_bwd(dy, w2, aux, dpre, bg), flush=True)


def t(fn, it=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it * 1e3


print("fused fwd us", t(lambda: C.linear_gelu_fwd(x, w1, b1, act, aux)))
print("plain fc1 us", t(lambda: torch.nn.functional.linear(x, w1)))
print("fused bwd us", t(lambda: C.linear_dgelu_bwd(dy, w2, aux, dpre, bg)))
print("plain dgrad us", t(lambda: dy.matmul(w2)))
ref = torch.nn.functional.gelu(x.float() @ w1.float().t() + b1.float(), approximate="tanh")
print("fwd max err", (act.float() - ref).abs().max().item())
