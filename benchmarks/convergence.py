#!/usr/bin/env python3
"""Training-curve check of the whole MI355X stack against PyTorch reference ops on the same GPU.

Single-step numerics tests (tests/test_model_gpu.py) compare one forward / backward with an fp32
reference; this runs the headline model (GPT-2 345M: 24 layers, h 1024, 16 heads, seq 1024) for
hundreds of Adam steps on LEARNABLE synthetic data and records the loss curve twice:

* ``--kernels 1``: the framework's path (flash attention forward / backward, fused
  bias-dropout-add-LayerNorm, fc1 + bias-GeLU and fc2-dgrad + GeLU-backward GEMM epilogues, the
  grouped MFMA weight-gradient kernel, fused LM-head cross-entropy, hand-written Adam);
* ``--kernels 0``: ``SMDT_DISABLE_KERNELS=1``, every op of the same model through its PyTorch
  reference on the same GPU (unfused attention, F.layer_norm, torch GEMMs, torch CE / Adam).

Same seed, same init, same batches, dropout off (the two paths draw their masks differently), so
the curves must track each other; a wrong gradient anywhere shows up as a diverging curve long
before it would show up in a one-step tolerance.

Data: a first-order Markov chain over 4096 token ids, every id with 4 fixed random successors
chosen uniformly — the achievable loss is ln 4 = 1.386 nats per token, far below the
uniform-vocabulary start (ln 50304 = 10.8), so the curve has somewhere to go. (No dataset is
downloadable here; the reference trains on CodeParrot)

Usage (GPU box): ``python benchmarks/convergence.py --kernels 1 --out k1.json`` and
``SMDT_DISABLE_KERNELS=1 python benchmarks/convergence.py --kernels 0 --out k0.json``, then
``python benchmarks/convergence.py --compare k1.json k0.json``.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import socket
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def markov_batches(steps: int, mbs: int, seq: int, states: int = 4096, fanout: int = 4, seed: int = 7):
    """[steps, mbs, seq + 1] int64 token ids of the chain (deterministic)."""
    rng = np.random.default_rng(seed)
    succ = rng.integers(0, states, size=(states, fanout))
    n = steps * mbs
    out = np.empty((n, seq + 1), dtype=np.int64)
    cur = rng.integers(0, states, size=n)
    out[:, 0] = cur
    for t in range(1, seq + 1):
        cur = succ[cur, rng.integers(0, fanout, size=n)]
        out[:, t] = cur
    return out.reshape(steps, mbs, seq + 1)


def train(a) -> dict:
    import torch
    from smdt_amd.comm import init_distributed
    from smdt_amd.models.gpt import GPTModel
    from smdt_amd.models.transformer import TransformerConfig
    from smdt_amd.optim.optimizer import MixedPrecisionAdam
    from smdt_amd.parallel import state as ps
    from smdt_amd.parallel.distributed import DistributedDataParallel
    from smdt_amd.ops import _ext

    for k, v in (("MASTER_ADDR", "127.0.0.1"), ("RANK", "0"), ("WORLD_SIZE", "1"), ("LOCAL_RANK", "0")):
        os.environ.setdefault(k, v)
    if "MASTER_PORT" not in os.environ:
        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            os.environ["MASTER_PORT"] = str(s.getsockname()[1])
    init_distributed("nccl")
    ps.initialize_model_parallel(1, 1)
    dev = torch.device("cuda", 0)
    if a.kernels:
        assert not _ext.kernels_disabled(), "--kernels 1 with SMDT_DISABLE_KERNELS=1"
        _ext.ext()     # fail loudly without the HIP extension
    else:
        assert _ext.kernels_disabled(), "--kernels 0 needs SMDT_DISABLE_KERNELS=1 in the environment"
    torch.manual_seed(1234)
    cfg = TransformerConfig(num_layers=a.layers, hidden_size=a.hidden, num_attention_heads=a.heads,
                            padded_vocab_size=50304, max_position_embeddings=a.seq, hidden_dropout=0.0,
                            attention_dropout=0.0, params_dtype=torch.bfloat16, seed=1234,
                            use_flash_attn=bool(a.kernels))
    model = GPTModel(cfg, device=dev)
    ddp = DistributedDataParallel(model, grad_dtype=torch.float32)
    opt = MixedPrecisionAdam(ddp, lr=a.lr, weight_decay=0.01, clip_grad=1.0, betas=(0.9, 0.95))
    data = torch.from_numpy(markov_batches(a.steps, a.mbs, a.seq))
    losses, t0 = [], time.time()
    for step in range(a.steps):
        lr = a.lr * min(1.0, (step + 1) / a.warmup)
        opt.set_lr(lr)
        tok = data[step].to(dev, non_blocking=True)
        ddp.zero_grad_buffer()
        loss = model(tok[:, :-1], labels=tok[:, 1:]).float().mean()
        loss.backward()
        ddp.finish_grad_sync()
        opt.step()
        losses.append(loss.item())
        if step % 50 == 0 or step == a.steps - 1:
            print(f"[conv] kernels={a.kernels} step {step} loss {losses[-1]:.4f} ({time.time() - t0:.0f}s)", flush=True)
    return {"kernels": a.kernels, "losses": losses, "config": vars(a),
            "wall_s": round(time.time() - t0, 1)}


def compare(p1: str, p0: str, label0: str = "PyTorch reference ops") -> str:
    k1 = json.load(open(p1))["losses"]
    k0 = json.load(open(p0))["losses"]
    n = min(len(k1), len(k0))
    d = np.abs(np.array(k1[:n]) - np.array(k0[:n]))
    tail = slice(max(0, n - 100), n)
    lines = [
        f"| quantity | HIP kernels | {label0} |",
        "|---|---|---|",
        f"| loss at step 0 | {k1[0]:.4f} | {k0[0]:.4f} |",
        f"| loss at step {n // 4} | {k1[n // 4]:.4f} | {k0[n // 4]:.4f} |",
        f"| loss at step {n // 2} | {k1[n // 2]:.4f} | {k0[n // 2]:.4f} |",
        f"| final loss (step {n - 1}) | {k1[n - 1]:.4f} | {k0[n - 1]:.4f} |",
        f"| mean loss, last 100 steps | {np.mean(k1[tail]):.4f} | {np.mean(k0[tail]):.4f} |",
        "",
        f"max |difference| over all {n} steps: {d.max():.4f} (step {int(d.argmax())}); mean over the last 100: "
        f"{d[tail].mean():.4f}; achievable loss ln 4 = {math.log(4):.4f}",
    ]
    return "\n".join(lines) + "\n"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kernels", type=int, default=1)
    ap.add_argument("--layers", type=int, default=24)
    ap.add_argument("--hidden", type=int, default=1024)
    ap.add_argument("--heads", type=int, default=16)
    ap.add_argument("--seq", type=int, default=1024)
    ap.add_argument("--mbs", type=int, default=8)
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--warmup", type=int, default=40)
    ap.add_argument("--lr", type=float, default=3e-4)
    ap.add_argument("--out", default=None)
    ap.add_argument("--compare", nargs=2, default=None, metavar=("KERNELS_JSON", "REFERENCE_JSON"))
    ap.add_argument("--label", default="PyTorch reference ops", help="column name of the second run")
    a = ap.parse_args()
    if a.compare:
        print(compare(*a.compare, label0=a.label))
        return
    res = train(a)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f)


if __name__ == "__main__":
    main()
