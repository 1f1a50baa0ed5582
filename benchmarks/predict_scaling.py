#!/usr/bin/env python3
"""Predicted bench.py step time at N = 2 / 4 / 8 GPUs from ONE MI355X plus the xGMI link budget.

The pool this repo is developed on has one GPU per box, so the multi-GPU points of the headline
(BASELINE.json: tokens/s of GPT-2 345M at 1/2/4/8 GPUs) are predicted before the driver measures
them. Two inputs:

(a) per-rank compute, MEASURED on one GPU by running bench.py on the shape one rank of each layout
    executes:
      * DP-N (N = 2 / 4, the default): every rank runs the whole model on its 64 sequences — the
        1-GPU step itself;
      * tp2 pp2 dp2 (N = 8, BASELINE): a rank holds 12 of the 24 layers with half the heads (8 x 64)
        and half the FFN (2048), and the last stage half of the (tied) LM head (vocab 50304 / 2);
        the replica's 4 GPUs process 4 x 64 = 256 sequences per step, as 8 micro-batches of 32.
        Emulated as a 12-layer model of that width on 256 sequences (micro-batch 32, 8
        micro-batches). Sequence parallelism would halve LayerNorm / dropout / residual work and
        the ring-chunked GEMMs run at M = 8192 instead of 16384: both are noted, not modelled;
      * tp2 (N = 2, the old default, ``--layout tp``): 24 layers at half width, 128 sequences.
(b) the link budget: ``LINK_GBPS`` per direction per xGMI link (MI355X: 7 links per GPU, every
    GPU pair directly connected), which of the step's bytes can hide behind compute (bucketed
    reduce-scatter during backward, parameter all-gather during the next forward, ring TP exchanges
    beside their chunk GEMMs, async pipeline p2p) and which cannot (the last gradient bucket, the
    tied-embedding all-reduce, the 1F1B bubble (pp - 1) / m, a link-bound TP exchange).

Usage (GPU box): ``python benchmarks/predict_scaling.py --out profiles/r3_predict`` runs the three
measurements and writes ``predicted.json`` + ``predicted.md``. ``--from-json`` recomputes the
table from saved measurements.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LINK_GBPS = 64.0            # per direction per xGMI link, conservative end of 64-77 (docs/XGMI.md)
H, L, S, V = 1024, 24, 1024, 50304
PARAMS = 354.9e6            # GPT-2 345M with the padded vocab (tied embedding)

_TP2 = ["--num-attention-heads", "8", "--kv-channels", "64", "--ffn-hidden-size", "2048", "--vocab-size", str(V // 2)]
_MB16 = ["--seqs-per-gpu", "256", "--micro-batch-size", "32", "--grad-accum", "8"]   # bench.py's N = 8 split
RUNS = {
    "n1_dp": [],
    # even split: 12 + 12 layers, the last stage also runs the LM head (the heavier stage)
    "tp2pp2_rank": ["--num-layers", "12"] + _TP2 + _MB16,
    # bench.py's balanced split (balanced_last_stage_layers): 13 layers | 11 layers + LM head
    "tp2pp2_stage0_bal": ["--num-layers", "13", "--emulate-first-stage"] + _TP2 + _MB16,
    "tp2pp2_stage1_bal": ["--num-layers", "11"] + _TP2 + _MB16,
    "tp2_rank": ["--num-attention-heads", "8", "--kv-channels", "64", "--ffn-hidden-size", "2048",
                 "--vocab-size", str(V // 2), "--seqs-per-gpu", "128", "--micro-batch-size", "64",
                 "--grad-accum", "2"],
}


def measure(steps: int, warmup: int, logdir: str) -> dict:
    out = {}
    for name, extra in RUNS.items():
        cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", str(steps), "--warmup", str(warmup),
               "--comm-stats", "1"] + extra
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=900, cwd=ROOT)
        with open(os.path.join(logdir, f"{name}.log"), "w") as f:
            f.write(r.stdout + "\n" + r.stderr)
        if r.returncode != 0:
            raise SystemExit(f"{name} failed:\n{r.stderr[-2000:]}")
        rec = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
        out[name] = {"ms_per_step": rec["ms_per_step"], "phase_ms": rec.get("phase_ms"),
                     "tokens_per_step": rec["config"]["global_batch"] * rec["config"]["seq_len"], "args": extra}
        print(f"[predict] {name}: {rec['ms_per_step']:.1f} ms", flush=True)
    return out


def link_ms(nbytes: float, links: float = 1.0) -> float:
    return nbytes / (LINK_GBPS * 1e9 * links) * 1e3


def predict(m: dict) -> list:
    rows = []
    t1 = m["n1_dp"]["ms_per_step"]
    tok1 = m["n1_dp"]["tokens_per_step"]
    rows.append({"N": 1, "layout": "tp1pp1dp1", "compute_ms": t1, "exposed_comm_ms": 0.0, "bubble_ms": 0.0,
                 "predicted_ms": t1, "tokens_per_step": tok1, "note": "measured"})
    # DP-N + ZeRO-1: fp32 gradient reduce-scatter + bf16 parameter all-gather, bucketed (16 MB).
    for n in (2, 4):
        links = n - 1                       # a direct reduce-scatter / all-gather uses every peer link
        rs = 4 * PARAMS * (n - 1) / n       # bytes each rank sends
        ag = 2 * PARAMS * (n - 1) / n
        hidden = link_ms(rs, links) + link_ms(ag, links)
        exposed = link_ms(16e6 * (n - 1) / n, links) + link_ms(2 * 16e6 / 4 * (n - 1) / n, links) + 0.3
        rows.append({"N": n, "layout": f"tp1pp1dp{n}+zero1", "compute_ms": t1, "exposed_comm_ms": round(exposed, 2),
                     "bubble_ms": 0.0, "predicted_ms": round(t1 + exposed, 1), "tokens_per_step": tok1 * n,
                     "note": f"{hidden:.1f} ms of RS+AG per step overlapped with backward / next forward"})
    # tp2 pp2 dp2 + SP (BASELINE at N = 8), with bench.py's balanced 13 | 11 split when measured.
    tr_even = m["tp2pp2_rank"]["ms_per_step"]
    bal = "tp2pp2_stage0_bal" in m and "tp2pp2_stage1_bal" in m
    tr = max(m["tp2pp2_stage0_bal"]["ms_per_step"], m["tp2pp2_stage1_bal"]["ms_per_step"]) if bal else tr_even
    mb, pp = 8, 2                                           # micro-batches per step, stages
    bubble = tr * (pp - 1) / mb
    grads = 4 * PARAMS / 4                                  # fp32 grads of a rank's quarter
    dp_tail = link_ms(16e6 / 2) + link_ms(8e6 / 2)          # last RS bucket + first AG bucket, dp2 = 1 link
    embd = link_ms(4 * (V // 2) * H)                        # tied-embedding grad all-reduce, first <-> last stage
    tp_chunk = S // 2 * 32 * H * 2                          # [s/2, mbs, h] bf16 = 32 MB per ring step
    relay_links = 4.0                                       # relay on 8 GPUs: ~4x one link (docs/XGMI.md)
    tp_per_ex = link_ms(tp_chunk, relay_links)
    tp_total = tp_per_ex * 8 * 12 * mb                      # 8 exchanges / layer / micro-batch, 12 layers
    exposed = dp_tail + embd + 0.5
    if bal:
        rows.append({"N": 8, "layout": "tp2pp2dp2+sp+zero1, even 12|12 split", "compute_ms": tr_even,
                     "exposed_comm_ms": round(exposed, 2), "bubble_ms": round(tr_even * (pp - 1) / mb, 1),
                     "predicted_ms": round(tr_even * (1 + (pp - 1) / mb) + exposed, 1), "tokens_per_step": tok1 * 8,
                     "note": "the last stage carries 12 layers + the LM head (2x the per-GPU head work of N = 1)"})
    rows.append({"N": 8, "layout": "tp2pp2dp2+sp+zero1" + (", split 13|11" if bal else ""), "compute_ms": tr,
                 "exposed_comm_ms": round(exposed, 2),
                 "bubble_ms": round(bubble, 1), "predicted_ms": round(tr + bubble + exposed, 1),
                 "tokens_per_step": tok1 * 8,
                 "note": (f"TP: {tp_total:.0f} ms of relayed exchanges ({tp_per_ex * 1e3:.0f} us each) beside "
                          f"chunk GEMMs; DP: {link_ms(grads / 2) + link_ms(grads / 4):.1f} ms RS+AG overlapped; "
                          f"SP halves LN/dropout work (not modelled)")})
    # the old N = 2 default, for the record: tp2 over ONE link
    t2 = m["tp2_rank"]["ms_per_step"]
    ex = S // 2 * 64 * H * 2                                # [s/2, 64, h] bf16 = 64 MB
    tp_total2 = link_ms(ex) * 8 * 24 * 2                    # 24 layers, 2 micro-batches of 64
    rows.append({"N": 2, "layout": "tp2+sp (--layout tp)", "compute_ms": t2,
                 "exposed_comm_ms": round(max(0.0, tp_total2 - t2), 1), "bubble_ms": 0.0,
                 "predicted_ms": round(max(t2, tp_total2), 1), "tokens_per_step": tok1 * 2,
                 "note": f"{tp_total2:.0f} ms of exchanges over the pair's single link: link-bound"})
    for r in rows:
        r["predicted_tokens_per_s"] = round(r["tokens_per_step"] / r["predicted_ms"] * 1e3)
        r["efficiency_vs_n1"] = round(r["predicted_tokens_per_s"] / (rows[0]["predicted_tokens_per_s"] * r["N"]), 3)
    return rows


def to_md(rows: list) -> str:
    lines = ["| N | layout | per-rank compute ms | 1F1B bubble ms | exposed comm ms | predicted ms/step | "
             "predicted tokens/s | efficiency vs N=1 | notes |", "|---|---|---|---|---|---|---|---|---|"]
    for r in rows:
        lines.append(f"| {r['N']} | {r['layout']} | {r['compute_ms']:.1f} | {r['bubble_ms']} | {r['exposed_comm_ms']} | "
                     f"{r['predicted_ms']} | {r['predicted_tokens_per_s'] / 1e3:.1f} k | {r['efficiency_vs_n1']:.2f} | "
                     f"{r['note']} |")
    return "\n".join(lines) + "\n"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "predict"))
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--from-json", default=None)
    a = ap.parse_args()
    os.makedirs(a.out, exist_ok=True)
    if a.from_json:
        with open(a.from_json) as f:
            m = json.load(f)["measured"]
    else:
        m = measure(a.steps, a.warmup, a.out)
    rows = predict(m)
    with open(os.path.join(a.out, "predicted.json"), "w") as f:
        json.dump({"measured": m, "link_GBps_per_direction": LINK_GBPS, "rows": rows}, f, indent=1)
    md = to_md(rows)
    with open(os.path.join(a.out, "predicted.md"), "w") as f:
        f.write(md)
    print(md)


if __name__ == "__main__":
    main()
