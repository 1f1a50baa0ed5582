"""Event simulation of the pipeline schedules of ``train/schedules.py`` — the per-rank issue order
of forward (F), input-gradient backward (B) and weight-gradient (W) work, with the cross-stage
dependencies of the p2p activations / gradients — for predicting the step time of a layout from
per-stage F / B / W times measured on ONE GPU (benchmarks/predict_scaling.py).

Model: each rank runs its ops in order on one stream (the compute stream); an op starts when the
previous op of its rank has finished and its input has arrived: F of micro-batch k on stage s
needs F_k of stage s-1 plus ``p2p`` ms; B_k on stage s needs B_k of stage s+1 plus ``p2p`` (the last
stage: its own F_k). W_k needs B_k of the same rank. A send is issued right after the op that
produces it, except in the ``1f1b`` schedule, where a stage's backward is one fused B+W op (the
weight-gradient GEMMs run inside backward, before the input gradient is sent).

Schedules (``train/schedules.py`` names):

* ``1f1b``     — Megatron's non-interleaved 1F1B; B and W fused, send after both.
* ``zb``       — the same order with the backward split (zero-bubble style, "B-send-W"): the input
                 gradient leaves after B, the stage's W GEMMs run while it travels.
* ``zbh1``     — ``zb`` plus, on rank r, the W of its last ``r + 1`` backward passes deferred behind
                 its LAST B: the last stages' final B passes, which every earlier stage waits for
                 in its cooldown, are not held up by W work, and that W work then runs while the
                 earlier stages finish (ZB-H1's idea, Qi et al., "Zero Bubble Pipeline
                 Parallelism", 2023: same activation memory as 1F1B, bubble ~ (pp-1)(F+B-W)).
* ``zbh2``     — ZB-H2-style: rank r runs 2 (pp - r - 1) forwards ahead (twice 1F1B's in-flight
                 micro-batches: the later stages never wait for an input after the first) and
                 defers the W of its last 2 (r + 1) passes. Activation memory on stage r grows to
                 2 (pp - r) - 1 micro-batches — free on a 288 GB MI355X (GPT-2 345M at tp2: ~1.6 GB
                 per in-flight micro-batch). At the BASELINE tp2pp2 point the bubble drops to the
                 first forward + hop that the last stage cannot avoid (16.2 -> 9.6 ms); with
                 m <= pp micro-batches it loses to zbh1.
"""
from __future__ import annotations

from typing import Dict, List, Sequence, Tuple

SCHEDULES = ("1f1b", "zb", "zbh1", "zbh2")


def warmup_and_defer(schedule: str, pp: int, r: int, m: int) -> Tuple[int, int]:
    """(forwards rank r runs before its first backward, first backward pass whose W is deferred
    behind the rank's last B) — shared with train/schedules.py so the simulation and the real
    schedule issue the same order."""
    if schedule == "zbh2":
        return min(2 * (pp - r - 1), m), max(0, m - 2 * (r + 1))
    warm = min(pp - r - 1, m)
    return warm, (max(0, m - (r + 1)) if schedule == "zbh1" else m)


def rank_ops(schedule: str, pp: int, r: int, m: int) -> List[Tuple[str, int]]:
    """The op sequence rank ``r`` issues: ("F", k), ("B", k), ("W", k) or ("BW", k) (1f1b)."""
    if schedule not in SCHEDULES:
        raise ValueError(f"unknown schedule {schedule!r}")
    warm, defer_from = warmup_and_defer(schedule, pp, r, m)
    steady = m - warm
    ops: List[Tuple[str, int]] = [("F", k) for k in range(warm)]
    fk, bk = warm, 0
    deferred: List[int] = []

    def backward(k):
        if schedule == "1f1b":
            ops.append(("BW", k))
            return
        ops.append(("B", k))
        if k >= defer_from:
            deferred.append(k)
        else:
            ops.append(("W", k))
    for i in range(steady):
        ops.append(("F", fk))
        fk += 1
        backward(bk)
        bk += 1
    for _ in range(warm):
        backward(bk)
        bk += 1
    ops.extend(("W", k) for k in deferred)
    return ops


def simulate(schedule: str, pp: int, m: int, F: Sequence[float], B: Sequence[float], W: Sequence[float],
             p2p: float = 0.0) -> Dict[str, object]:
    """Makespan (ms) of one pipelined step. ``F[s]``, ``B[s]``, ``W[s]``: per-micro-batch times of
    stage s (B: input-gradient backward alone; W: its weight-gradient GEMMs). Returns the makespan,
    each rank's finish time and idle time, and the bubble = makespan - max busy time."""
    ops = [rank_ops(schedule, pp, r, m) for r in range(pp)]
    pos = [0] * pp
    t_rank = [0.0] * pp
    done: Dict[Tuple[str, int, int], float] = {}   # (kind, stage, k) -> finish time

    def ready(r, kind, k):
        if kind == "F":
            return 0.0 if r == 0 else done.get(("F", r - 1, k))
        if kind in ("B", "BW"):
            if r == pp - 1:
                return done.get(("F", r, k))
            key = ("B", r + 1, k)
            return done.get(key)
        if kind == "W":
            return done.get(("B", r, k))
        raise ValueError(kind)

    total = sum(len(o) for o in ops)
    finished = 0
    while finished < total:
        progressed = False
        for r in range(pp):
            while pos[r] < len(ops[r]):
                kind, k = ops[r][pos[r]]
                dep = ready(r, kind, k)
                if dep is None:
                    break
                lat = p2p if (kind == "F" and r > 0) or (kind in ("B", "BW") and r < pp - 1) else 0.0
                start = max(t_rank[r], dep + lat)
                cost = {"F": F[r], "B": B[r], "W": W[r], "BW": B[r] + W[r]}[kind]
                end = start + cost
                t_rank[r] = end
                if kind == "BW":
                    done[("B", r, k)] = end        # the gradient leaves after the fused B + W
                    done[("W", r, k)] = end
                else:
                    done[(kind, r, k)] = end
                pos[r] += 1
                finished += 1
                progressed = True
        if not progressed:
            raise RuntimeError(f"schedule {schedule} deadlocks (pp {pp}, m {m})")
    busy = [m * (F[r] + B[r] + W[r]) for r in range(pp)]
    span = max(t_rank)
    return {"makespan": span, "finish": t_rank, "idle": [span - b for b in busy],
            "bubble": span - max(busy)}
