#!/usr/bin/env python3
"""Predicted bench.py step time at N = 2 / 4 / 8 GPUs from ONE MI355X plus the xGMI link budget.

The pool this repo is developed on has one GPU per box, so the multi-GPU points of the headline
(BASELINE.json: tokens/s of GPT-2 345M at 1/2/4/8 GPUs) and the GPT-3 6.7B TP4 PP2 + SP layout
(BASELINE config #5) are predicted before the driver measures them. Inputs:

(a) per-rank compute, MEASURED on one GPU by running bench.py on exactly what one rank executes:
      * DP-N (N = 2 / 4, the default): the 1-GPU step itself (every rank runs the whole model);
      * tp2 pp2 dp2 + SP (N = 8, BASELINE): ``bench.py --emulate-tp 2`` — ONE process as TP rank 0
        (parallel/state.initialize_emulated_tensor_parallel, comm/loopback.py): the sharded heads /
        FFN / vocab, sequence-parallel LayerNorm / dropout on s/2 rows, the ring collective-matmul's
        per-chunk GEMMs at their real M = s/2 x mbs, the vocab-parallel head + CE; every collective
        is a local stand-in with the receiving side's memory traffic. One run
        per pipeline stage at bench.py's 13 | 11 split (first stage without the head, last stage
        with it and without the embedding: its input is a received activation), plus the even
        12 | 12 split the interleaved schedule needs;
      * GPT-3 6.7B tp4 pp2 + SP: the same with ``--emulate-tp 4``, 16 layers per stage, seq 2048,
        8 micro-batches of 4 (32 sequences per replica per step).
    Each emulated run also reports ``fbw_ms``: per micro-batch forward (F), input-gradient backward
    with the weight-gradient GEMMs held (B) and those GEMMs (W).
(b) the pipeline bubble of each schedule from train/pipeline_sim.simulate(F, B, W per stage, the
    p2p hop of one [s/tp, mbs, h] activation over one link) — 1F1B, the zero-bubble split zb and
    zbh1 and zbh2 (the bench default) — and the interleaved vpp = 2 schedule as 1F1B's bubble / 2 on the
    even split;
(c) the link budget: ``LINK_GBPS`` per direction per xGMI link (7 links per GPU, every pair directly
    connected): which of the step's bytes hide behind compute (bucketed reduce-scatter during
    backward, parameter all-gather during the next forward, TP exchanges beside their chunk GEMMs)
    and which cannot (the last gradient bucket, the tied-embedding all-reduce, a link-bound TP
    exchange).

Usage (GPU box): ``python benchmarks/predict_scaling.py --out profiles/r4_predict`` runs the
measurements and writes ``predicted.json`` + ``predicted.md``; ``--from-json`` recomputes the
tables from saved measurements (CPU).
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from smdt_amd.train.pipeline_sim import simulate  # noqa: E402

LINK_GBPS = 64.0            # per direction per xGMI link, conservative end of 64-77 (docs/XGMI.md)
H, L, S, V = 1024, 24, 1024, 50304
PARAMS = 354.9e6            # GPT-2 345M with the padded vocab (tied embedding)

_N8 = ["--emulate-tp", "2", "--micro-batch-size", "32", "--grad-accum", "8", "--phase-probe", "8"]
_N8_64 = ["--emulate-tp", "2", "--micro-batch-size", "64", "--grad-accum", "4", "--phase-probe", "4"]
# GPT-3 stage shapes: the committed TunableOp table has their winners (profiles/r6_g3tune/: 397.1 /
# 397.8 ms against 399.7 / 400.3 with the library heuristics)
_G3 = ["--emulate-tp", "4", "--hidden-size", "4096", "--num-attention-heads", "32", "--seq-length", "2048",
       "--micro-batch-size", "4", "--grad-accum", "8", "--phase-probe", "8"]
RUNS = {
    "n1_dp": [],
    # bench.py's balanced split: 13 layers | 11 layers + LM head
    "tp2pp2_stage0": ["--num-layers", "13", "--emulate-first-stage"] + _N8,
    "tp2pp2_stage1": ["--num-layers", "11", "--emulate-last-stage"] + _N8,
    # the even split the interleaved schedule is limited to: 12 | 12 + head (the heavier stage)
    "tp2pp2_stage1_even": ["--num-layers", "12", "--emulate-last-stage"] + _N8,
    # the same replica batch as 4 micro-batches of 64: ring chunks of 32768 rows (the N = 1 GEMM
    # shapes, half the launches) against twice the bubble per micro-batch
    "tp2pp2_mb64_stage0": ["--num-layers", "13", "--emulate-first-stage"] + _N8_64,
    "tp2pp2_mb64_stage1": ["--num-layers", "11", "--emulate-last-stage"] + _N8_64,
    "gpt3_tp4_stage0": ["--num-layers", "16", "--emulate-first-stage"] + _G3,
    "gpt3_tp4_stage1": ["--num-layers", "16", "--emulate-last-stage"] + _G3,
    # the whole 6.7B model on ONE GPU (288 GB hold weights, fp32 masters, Adam state, activations)
    "gpt3_n1": ["--hidden-size", "4096", "--num-attention-heads", "32", "--seq-length", "2048", "--num-layers", "32",
                "--micro-batch-size", "4", "--grad-accum", "1", "--tunableop", "0"],
}
# the N = 8 stage ranks with the TP exchanges MEASURED: the paced link stand-in (comm/loopback.py,
# SMDT_LINK_STANDIN=relay: the relay's modelled 131 us per 33.6 MB chunk and its 64 workgroups on a
# side stream beside the rank's compute) instead of an in-line copy; the stage times and F / B / W
# then include whatever of the exchanges the compute does not hide (profiles/r6_standin/).
# STANDIN_ENV holds the exchange-overlap settings the bench's N = 8 run uses.
STANDIN_ENV = {"SMDT_LINK_STANDIN": "relay", "SMDT_RING_GEMM_TN": "1", "SMDT_W_FILL": "1"}
RUNS["tp2pp2_stage0_standin"] = RUNS["tp2pp2_stage0"]
RUNS["tp2pp2_stage1_standin"] = RUNS["tp2pp2_stage1"]
# the same replica batch split differently, exchanges measured: 4 x 64 (bigger chunk GEMMs and
# exchanges, twice the bubble per micro-batch) and 16 x 16 (smaller ones, half the bubble)
_N8_16 = ["--emulate-tp", "2", "--micro-batch-size", "16", "--grad-accum", "16", "--phase-probe", "16"]
RUNS["tp2pp2_mb64_stage0_standin"] = RUNS["tp2pp2_mb64_stage0"]
RUNS["tp2pp2_mb64_stage1_standin"] = RUNS["tp2pp2_mb64_stage1"]
RUNS["tp2pp2_mb16_stage0_standin"] = ["--num-layers", "13", "--emulate-first-stage"] + _N8_16
RUNS["tp2pp2_mb16_stage1_standin"] = ["--num-layers", "11", "--emulate-last-stage"] + _N8_16
# GPT-3 tp4 stages with the SP exchanges MEASURED: TpDirect's row pieces over a paced stand-in of
# the direct engine (comm/loopback.PacedDirectEngine: 3 links at LINK_GBPS, 32 workgroups)
DIRECT_ENV = {"SMDT_LINK_STANDIN": f"direct:{LINK_GBPS:g}:32", "SMDT_RING_GEMM_TN": "1", "SMDT_W_FILL": "1"}
RUNS["gpt3_tp4_stage0_direct"] = RUNS["gpt3_tp4_stage0"]
RUNS["gpt3_tp4_stage1_direct"] = RUNS["gpt3_tp4_stage1"]
_COPY_ENV = {"SMDT_W_FILL": "0", "SMDT_RING_GEMM_TN": "0"}   # compute-only runs: no overlap machinery
RUN_ENV = {"tp2pp2_stage0_standin": STANDIN_ENV, "tp2pp2_stage1_standin": STANDIN_ENV,
           **{f"tp2pp2_mb{m}_stage{i}_standin": STANDIN_ENV for m in (16, 64) for i in (0, 1)},
           "gpt3_tp4_stage0_direct": DIRECT_ENV, "gpt3_tp4_stage1_direct": DIRECT_ENV,
           **{k: _COPY_ENV for k in ("tp2pp2_stage0", "tp2pp2_stage1", "tp2pp2_stage1_even",
                                     "tp2pp2_mb64_stage0", "tp2pp2_mb64_stage1")}}
SCHEDS = ("1f1b", "zb", "zbh1", "zbh2")


def measure(steps: int, warmup: int, logdir: str, only=None) -> dict:
    out = {}
    for name, extra in RUNS.items():
        if only and name not in only:
            continue
        cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", str(steps), "--warmup", str(warmup),
               "--comm-stats", "1"] + extra
        env = dict(os.environ, **RUN_ENV.get(name, {}))
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=900, cwd=ROOT, env=env)
        with open(os.path.join(logdir, f"{name}.log"), "w") as f:
            f.write(r.stdout + "\n" + r.stderr)
        if r.returncode != 0:
            raise SystemExit(f"{name} failed:\n{r.stderr[-2000:]}")
        rec = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
        out[name] = {"ms_per_step": rec["ms_per_step"], "phase_ms": rec.get("phase_ms"), "fbw_ms": rec.get("fbw_ms"),
                     "tokens_per_step": rec["config"]["global_batch"] * rec["config"]["seq_len"], "args": extra}
        print(f"[predict] {name}: {rec['ms_per_step']:.1f} ms  fbw {rec.get('fbw_ms')}", flush=True)
    return out


def link_ms(nbytes: float, links: float = 1.0) -> float:
    return nbytes / (LINK_GBPS * 1e9 * links) * 1e3


def _fbw(m, name):
    d = m[name]["fbw_ms"]
    return d["F"], d["B"], d["W"]


def pipeline_rows(m, st0, st1, mb, pp, act_bytes, exposed, tok, label, even=None):
    """One row per schedule for a pp = 2 layout from the two measured stages."""
    rows = []
    t = [m[st0]["ms_per_step"], m[st1]["ms_per_step"]]
    f0, b0, w0 = _fbw(m, st0)
    f1, b1, w1 = _fbw(m, st1)
    hop = link_ms(act_bytes)
    for sched in SCHEDS:
        sim = simulate(sched, pp, mb, [f0, f1], [b0, b1], [w0, w1], p2p=hop)
        bubble = sim["bubble"]
        pred = max(t) + bubble + exposed
        rows.append({"layout": f"{label}, {sched}", "compute_ms": round(max(t), 1),
                     "stage_ms": [round(x, 1) for x in t], "bubble_ms": round(bubble, 1),
                     "exposed_comm_ms": round(exposed, 2), "predicted_ms": round(pred, 1),
                     "tokens_per_step": tok,
                     "note": f"F/B/W per micro-batch: stage 0 {f0:.2f}/{b0:.2f}/{w0:.2f}, stage 1 {f1:.2f}/{b1:.2f}/{w1:.2f} ms; "
                             f"p2p hop {hop:.2f} ms"})
    if even is not None:
        te = [m[st0]["ms_per_step"] * 12.0 / 13.0, m[even]["ms_per_step"]]   # 12 | 12 + head
        fe, be, we = _fbw(m, even)
        sim = simulate("1f1b", pp, mb, [f0 * 12 / 13, fe], [b0 * 12 / 13, be], [w0 * 12 / 13, we], p2p=hop)
        bubble = sim["bubble"] / 2.0
        pred = max(te) + bubble + exposed
        rows.append({"layout": f"{label}, interleaved vpp2 (even 12|12 split)", "compute_ms": round(max(te), 1),
                     "stage_ms": [round(x, 1) for x in te], "bubble_ms": round(bubble, 1),
                     "exposed_comm_ms": round(exposed, 2), "predicted_ms": round(pred, 1), "tokens_per_step": tok,
                     "note": "1F1B bubble / vpp; uniform layer split only (the LM head stage carries 12 layers)"})
    return rows


def predict(m: dict) -> list:
    rows = []
    t1 = m["n1_dp"]["ms_per_step"]
    tok1 = m["n1_dp"]["tokens_per_step"]
    rows.append({"N": 1, "model": "gpt2-345m", "layout": "tp1pp1dp1", "compute_ms": t1, "exposed_comm_ms": 0.0,
                 "bubble_ms": 0.0, "predicted_ms": t1, "tokens_per_step": tok1, "note": "measured"})
    # DP-N + ZeRO-1: fp32 gradient reduce-scatter + bf16 parameter all-gather, bucketed (16 MB)
    for n in (2, 4):
        links = n - 1                       # a direct reduce-scatter / all-gather uses every peer link
        rs = 4 * PARAMS * (n - 1) / n       # bytes each rank sends
        ag = 2 * PARAMS * (n - 1) / n
        hidden = link_ms(rs, links) + link_ms(ag, links)
        exposed = link_ms(16e6 * (n - 1) / n, links) + link_ms(2 * 16e6 / 4 * (n - 1) / n, links) + 0.3
        rows.append({"N": n, "model": "gpt2-345m", "layout": f"tp1pp1dp{n}+zero1", "compute_ms": t1,
                     "exposed_comm_ms": round(exposed, 2), "bubble_ms": 0.0, "predicted_ms": round(t1 + exposed, 1),
                     "tokens_per_step": tok1 * n,
                     "note": f"{hidden:.1f} ms of RS+AG per step overlapped with backward / next forward"})
    # N = 8: tp2 pp2 dp2 + SP + ZeRO-1 (BASELINE config #3)
    dp_tail = link_ms(16e6 / 2) + link_ms(8e6 / 2)              # last RS bucket + first AG bucket, dp2 = 1 link
    embd = link_ms(4 * (V // 2) * H)                            # tied-embedding fp32 grad all-reduce, 1 link
    if "tp2pp2_stage0" in m and "tp2pp2_stage1" in m:
        act = (S // 2) * 32 * H * 2                             # p2p activation [s/2, 32, h] bf16
        for r in pipeline_rows(m, "tp2pp2_stage0", "tp2pp2_stage1", 8, 2, act, dp_tail + embd + 0.5, tok1 * 8,
                               "tp2pp2dp2+sp+zero1 13|11", even="tp2pp2_stage1_even" if "tp2pp2_stage1_even" in m else None):
            rows.append({"N": 8, "model": "gpt2-345m", **r})
        rows += gpt2_tp2_exchange_rows(m, act, dp_tail + embd + 0.5, tok1 * 8)
    if "tp2pp2_stage0_standin" in m and "tp2pp2_stage1_standin" in m:
        act = (S // 2) * 32 * H * 2
        flags = " ".join(f"{k}={v}" for k, v in STANDIN_ENV.items() if k != "SMDT_LINK_STANDIN")
        for r in pipeline_rows(m, "tp2pp2_stage0_standin", "tp2pp2_stage1_standin", 8, 2, act,
                               dp_tail + embd + 0.5, tok1 * 8,
                               f"tp2pp2dp2+sp+zero1 13|11, TP exchanges MEASURED (paced relay stand-in; {flags})"):
            if r["layout"].endswith("zbh2"):
                rows.append({"N": 8, "model": "gpt2-345m", **r})
    for mbs, nmb in ((64, 4), (16, 16)):
        k0, k1 = f"tp2pp2_mb{mbs}_stage0_standin", f"tp2pp2_mb{mbs}_stage1_standin"
        if k0 in m and k1 in m:
            actm = (S // 2) * mbs * H * 2
            for r in pipeline_rows(m, k0, k1, nmb, 2, actm, dp_tail + embd + 0.5, tok1 * 8,
                                   f"tp2pp2dp2+sp+zero1 13|11, {nmb} x {mbs}, TP exchanges MEASURED (paced relay stand-in)"):
                if r["layout"].endswith("zbh2"):
                    rows.append({"N": 8, "model": "gpt2-345m", **r})
    if "tp2pp2_mb64_stage0" in m and "tp2pp2_mb64_stage1" in m:
        act64 = (S // 2) * 64 * H * 2
        for r in pipeline_rows(m, "tp2pp2_mb64_stage0", "tp2pp2_mb64_stage1", 4, 2, act64, dp_tail + embd + 0.5,
                               tok1 * 8, "tp2pp2dp2+sp+zero1 13|11, 4 x 64"):
            rows.append({"N": 8, "model": "gpt2-345m", **r})
    for r in rows:
        r["predicted_tokens_per_s"] = round(r["tokens_per_step"] / r["predicted_ms"] * 1e3)
        r["efficiency_vs_n1"] = round(r["predicted_tokens_per_s"] / (rows[0]["predicted_tokens_per_s"] * r["N"]), 3)
    return rows


def _ag_exposed(g: float, t_x: float, W: int, k: int, wq: float = 0.0) -> float:
    """Compute-stream time lost to an all-gather collective-matmul beyond its GEMMs (g ms over all
    W chunks) and the weight-gradient GEMMs drained before the last wait (wq): the transfer runs
    as k row pieces back to back on the engine stream (t_x ms in all); the local chunk's GEMM runs
    beside the first piece, the peers' rows of piece j once piece j has landed
    (comm/tp_direct.TpDirect.all_gather; the ring is k = W - 1 pieces of one chunk each, its
    local chunk first)."""
    piece = t_x / k
    c = g / W
    per = g * (W - 1) / (W * k)
    for j in range(k):
        if j == k - 1:
            c += wq
        c = max(c, (j + 1) * piece) + per
    return c - (g + wq)


def _rs_exposed(g: float, t_x: float, k: int, wq: float = 0.0) -> float:
    """The same for a reduce-scatter collective-matmul: piece j's partial GEMMs (g / k), then its
    reduce-scatter on the engine stream (t_x / k) beside piece j + 1's GEMMs; the queued
    weight-gradient GEMMs (wq) run before the last wait (TpDirect.reduce_scatter, ``rs_ring``)."""
    c = e = 0.0
    for _ in range(k):
        c += g / k
        e = max(e, c) + t_x / k
    c += wq
    return max(c, e) - (g + wq)


SYNC_MS = 0.012   # per-exchange cross-stream hand-off, eager (profiles/r5_lb_async_neg/: 10.5 ms / 869)


def _ring2_exposed(g: float, t_x: float, wq: float = 0.0) -> float:
    """A 2-rank ring collective-matmul (``ag_ring`` / ``rs_ring`` at tp = 2): the transfer (t_x)
    runs beside ONE of the two chunk GEMMs (g / 2) and, in backward, the weight-gradient GEMMs
    drained before the wait (wq)."""
    return max(0.0, t_x - g / 2 - wq)


def gpt2_tp2_exchange_model(W_mb_ms: float, layers: int, mb: int, t_x: float, sync_ms: float = SYNC_MS) -> dict:
    """Exposed SP-exchange time per step of one tp2 stage of the BASELINE N = 8 layout: per layer
    and micro-batch 8 exchanges (forward AG qkv / RS proj / AG fc1 / RS fc2; backward AG fc2 /
    RS fc1 / AG proj / RS qkv), each against its own chunk GEMMs priced from the stage's measured
    weight-gradient time per micro-batch (W / layers, split by FLOPs qkv 3 : proj 1 : fc1 4 :
    fc2 4), backward ones with their linear's wgrad as the drained queue; plus ``sync_ms`` per
    exchange for the side-stream hand-off the emulation does not pay (it copies in line)."""
    g = W_mb_ms / layers
    gl = {n: g * f for n, f in {"qkv": 3 / 12, "proj": 1 / 12, "fc1": 4 / 12, "fc2": 4 / 12}.items()}
    fwd = sum(_ring2_exposed(gl[n], t_x) for n in ("qkv", "proj", "fc1", "fc2"))
    bwd = sum(_ring2_exposed(gl[n], t_x, wq=gl[n]) for n in ("fc2", "fc1", "proj", "qkv"))
    per_step = layers * mb * (fwd + bwd + 8 * sync_ms)
    return {"fwd_per_layer_mb": fwd, "bwd_per_layer_mb": bwd, "exposed_ms": per_step}


def gpt2_tp2_exchange_rows(m: dict, act_bytes: float, other_exposed: float, tok: float) -> list:
    """The N = 8 zbh2 row again with the TP-pair exchanges SIMULATED instead of assumed hidden:
    one [s/2, 32, h] bf16 chunk per exchange, over the relay (every TP pair of the node exchanging
    at once: each directed link carries 2/8 of a message, W/2 = 4 links' worth, docs/XGMI.md) or,
    if the relay lost its start-up timing, over RCCL's single link. Each stage pays its own
    exposure; the slower stage sets the step."""
    names = ("tp2pp2_stage0", "tp2pp2_stage1")
    if not all(n in m and m[n].get("fbw_ms") for n in names):
        return []
    base = [r for r in pipeline_rows(m, names[0], names[1], 8, 2, act_bytes, other_exposed, tok,
                                     "tp2pp2dp2+sp+zero1 13|11") if r["layout"].endswith("zbh2")][0]
    ex_bytes = (S // 2) * 32 * H * 2
    rows = []
    for links, name in ((4.0, "relay, all 4 pairs at once"), (1.0, "RCCL p2p, one link")):
        # (layout keys: "... TP exchange relay" / "... TP exchange RCCL p2p"; the rest goes to the note)
        t_x = link_ms(ex_bytes, links)
        exp, notes = [], []
        for n, layers in zip(names, (13, 11)):
            mdl = gpt2_tp2_exchange_model(m[n]["fbw_ms"]["W"], layers, 8, t_x)
            exp.append(mdl["exposed_ms"])
            notes.append(f"fwd {mdl['fwd_per_layer_mb']:.3f} / bwd {mdl['bwd_per_layer_mb']:.3f}")
        stage = [m[n]["ms_per_step"] + e for n, e in zip(names, exp)]
        pred = max(stage) + base["bubble_ms"] + other_exposed
        rows.append({"N": 8, "model": "gpt2-345m", "layout": f"tp2pp2dp2+sp+zero1 13|11, zbh2, TP exchange {name.split(',')[0]}",
                     "compute_ms": base["compute_ms"], "stage_ms": base["stage_ms"], "bubble_ms": base["bubble_ms"],
                     "exposed_comm_ms": round(max(stage) - base["compute_ms"] + other_exposed, 1),
                     "predicted_ms": round(pred, 1), "tokens_per_step": tok,
                     "note": f"{name}: {t_x * 1e3:.0f} us per {ex_bytes / 1e6:.1f} MB exchange; exposed per layer and "
                             f"micro-batch (stage 0 ; stage 1) {' ; '.join(notes)} ms + {SYNC_MS * 1e3:.0f} us "
                             f"hand-off per exchange; stages with exposure {stage[0]:.1f} / {stage[1]:.1f} ms"})
    return rows


def gpt3_exchange_model(W_ms: float, layers: int, mb: int, t_x: float, tp: int, k: int) -> dict:
    """Exposed SP-exchange time per step for one tp4 stage: per layer and micro-batch the 8
    exchanges (forward AG qkv / RS proj / AG fc1 / RS fc2, backward AG fc2 / RS fc1 / AG proj /
    RS qkv) simulated against their own GEMMs, which are priced from the measured weight-gradient
    GEMM time of a micro-batch (``W`` of the stage's F/B/W split: the forward and the input-gradient
    GEMMs have the same FLOPs) split over the four linears by FLOPs (qkv 3, proj 1, fc1 4, fc2 4 of
    12 h^2); the backward's exchanges get their linear's weight-gradient GEMM as the drained queue.
    Plus the embedding output's reduce-scatter per micro-batch (no GEMM partner)."""
    g = W_ms / layers
    share = {"qkv": 3 / 12, "proj": 1 / 12, "fc1": 4 / 12, "fc2": 4 / 12}
    gl = {n: g * f for n, f in share.items()}
    fwd = (_ag_exposed(gl["qkv"], t_x, tp, k) + _rs_exposed(gl["proj"], t_x, k)
           + _ag_exposed(gl["fc1"], t_x, tp, k) + _rs_exposed(gl["fc2"], t_x, k))
    bwd = (_ag_exposed(gl["fc2"], t_x, tp, k, wq=gl["fc2"]) + _rs_exposed(gl["fc1"], t_x, k, wq=gl["fc1"])
           + _ag_exposed(gl["proj"], t_x, tp, k, wq=gl["proj"]) + _rs_exposed(gl["qkv"], t_x, k, wq=gl["qkv"]))
    per_step = layers * mb * (fwd + bwd) + mb * t_x
    return {"fwd_per_layer_mb": fwd, "bwd_per_layer_mb": bwd, "exposed_ms": per_step}


def predict_gpt3(m: dict) -> list:
    """GPT-3 6.7B, tp4 pp2 + SP on 8 GPUs (BASELINE config #5): per-rank compute from the emulated
    stages; the sequence-parallel exchanges per rank and step (8 per layer and micro-batch — the
    all-gathers before QKV and fc1 and the reduce-scatters after proj and fc2, forward, and their
    mirror images in backward (the gathered inputs are kept for the weight gradients, no re-gather)
    — plus the embedding's / LM head's 2 per micro-batch, each 3/4 of a [2048, 4, 4096] bf16
    activation) over ONE link per direction (the ring) or over the three links of the TP group (a
    direct exchange). The exposed part is SIMULATED per exchange against its own GEMMs
    (``gpt3_exchange_model``): the ring's chunk-by-chunk overlap, and the direct engine gathering /
    reducing whole chunks (1 piece: only the local chunk's GEMM beside the gather, every partial
    before the reduce-scatter — the round-4 engine) or in 2 / 4 row pieces (round 5,
    ``SMDT_TP_DIRECT_PIECES``)."""
    if not ("gpt3_tp4_stage0" in m and "gpt3_tp4_stage1" in m):
        return []
    rows = []
    sl, mb, h, layers, tp = 2048, 4, 4096, 16, 4
    xfer_bytes = 8 * (8 * layers + 2) * 0.75 * sl * mb * h * 2   # 8 micro-batches per step
    tok = 32 * sl                                           # tp4 x pp2 = 8 GPUs: ONE replica, 32 sequences
    act = (sl // 4) * mb * h * 2
    base = pipeline_rows(m, "gpt3_tp4_stage0", "gpt3_tp4_stage1", 8, 2, act, 0.0, tok, "tp4pp2dp1+sp")
    # the split-backward schedule with the lowest predicted step (zbh2 at these micro-batch counts)
    zbh1 = min((r for r in base if r["layout"].split(", ")[-1] in ("zbh1", "zbh2")), key=lambda r: r["predicted_ms"])
    sched = zbh1["layout"].split(", ")[-1]
    comp = zbh1["compute_ms"]
    slow = max(("gpt3_tp4_stage0", "gpt3_tp4_stage1"), key=lambda n: m[n]["ms_per_step"])
    W_ms = m[slow]["fbw_ms"]["W"]
    ex_bytes = 0.75 * sl * mb * h * 2                       # one exchange, per rank
    for links, k, name in ((1, tp - 1, "ring, one link per direction"),
                           (3, 1, "direct, 3 links, whole chunks (round 4)"),
                           (3, 2, "direct, 3 links, 2 row pieces"),
                           (3, 4, "direct, 3 links, 4 row pieces")):
        t_x = link_ms(ex_bytes, links)
        mdl = gpt3_exchange_model(W_ms, layers, 8, t_x, tp, k)
        exposed = mdl["exposed_ms"]
        pred = zbh1["predicted_ms"] + exposed
        rows.append({"N": 8, "model": "gpt3-6.7b", "layout": f"tp4pp2+sp, {sched}, TP exchange {name}",
                     "compute_ms": comp, "stage_ms": zbh1["stage_ms"], "bubble_ms": zbh1["bubble_ms"],
                     "exposed_comm_ms": round(exposed, 1), "predicted_ms": round(pred, 1), "tokens_per_step": tok,
                     "note": f"{xfer_bytes / 1e9:.1f} GB of SP exchanges per rank per step = "
                             f"{link_ms(xfer_bytes, links):.0f} ms on {links} link(s); exposed per layer and "
                             f"micro-batch fwd {mdl['fwd_per_layer_mb']:.3f} / bwd {mdl['bwd_per_layer_mb']:.3f} ms "
                             f"against {W_ms / layers:.3f} ms of GEMMs per pass"})
    if "gpt3_tp4_stage0_direct" in m and "gpt3_tp4_stage1_direct" in m:
        # the same layout with the exchanges MEASURED inside the emulated stages (no model term)
        flags = " ".join(f"{k}={v}" for k, v in DIRECT_ENV.items())
        for r in pipeline_rows(m, "gpt3_tp4_stage0_direct", "gpt3_tp4_stage1_direct", 8, 2, act, 0.0, tok,
                               f"tp4pp2+sp, TP exchanges MEASURED (paced direct-engine stand-in; {flags})"):
            if r["layout"].endswith(sched):
                rows.append({"N": 8, "model": "gpt3-6.7b", **r})
    return rows


def to_md(rows: list) -> str:
    lines = ["| N | model | layout | per-rank compute ms (stages) | bubble ms | exposed comm ms | predicted ms/step | "
             "predicted tokens/s | efficiency vs N=1 | notes |", "|---|---|---|---|---|---|---|---|---|---|"]
    for r in rows:
        stages = f" ({' / '.join(str(x) for x in r['stage_ms'])})" if r.get("stage_ms") else ""
        eff = f"{r['efficiency_vs_n1']:.2f}" if "efficiency_vs_n1" in r else "-"
        lines.append(f"| {r['N']} | {r['model']} | {r['layout']} | {r['compute_ms']:.1f}{stages} | {r['bubble_ms']} | "
                     f"{r['exposed_comm_ms']} | {r['predicted_ms']} | {r['predicted_tokens_per_s'] / 1e3:.1f} k | {eff} | "
                     f"{r['note']} |")
    return "\n".join(lines) + "\n"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "predict"))
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--only", nargs="*", default=None, help="measure only these runs")
    ap.add_argument("--from-json", default=None)
    ap.add_argument("--merge-json", default=None,
                    help="start from these saved measurements; --only re-measures and replaces runs")
    a = ap.parse_args()
    os.makedirs(a.out, exist_ok=True)
    if a.from_json:
        with open(a.from_json) as f:
            m = json.load(f)["measured"]
    else:
        m = {}
        if a.merge_json:
            with open(a.merge_json) as f:
                m = json.load(f)["measured"]
        m.update(measure(a.steps, a.warmup, a.out, a.only))
    rows = predict(m)
    g3 = predict_gpt3(m)
    for r in g3:
        r["predicted_tokens_per_s"] = round(r["tokens_per_step"] / r["predicted_ms"] * 1e3)
        if "gpt3_n1" in m:   # vs 8 GPUs each running the whole model data-parallel at N = 1's rate
            n1 = m["gpt3_n1"]["tokens_per_step"] / m["gpt3_n1"]["ms_per_step"] * 1e3
            r["efficiency_vs_n1"] = round(r["predicted_tokens_per_s"] / (8 * n1), 3)
    with open(os.path.join(a.out, "predicted.json"), "w") as f:
        json.dump({"measured": m, "link_GBps_per_direction": LINK_GBPS, "rows": rows, "gpt3_rows": g3}, f, indent=1)
    md = to_md(rows) + ("\n" + to_md(g3) if g3 else "")
    with open(os.path.join(a.out, "predicted.md"), "w") as f:
        f.write(md)
    print(md)


if __name__ == "__main__":
    main()
