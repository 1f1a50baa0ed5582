"""train/pipeline_sim.py: the schedules' per-rank op order and the simulated bubble (the model
benchmarks/predict_scaling.py prices the N = 8 pipeline with)."""
import pytest

from smdt_amd.train.pipeline_sim import SCHEDULES, rank_ops, simulate


@pytest.mark.parametrize("schedule", SCHEDULES)
@pytest.mark.parametrize("pp,m", [(2, 8), (4, 8), (4, 3)])
def test_rank_ops_cover_every_microbatch_once(schedule, pp, m):
    for r in range(pp):
        ops = rank_ops(schedule, pp, r, m)
        kinds = ("BW",) if schedule == "1f1b" else ("B", "W")
        assert sorted(k for kind, k in ops if kind == "F") == list(range(m))
        for kd in kinds:
            assert sorted(k for kind, k in ops if kind == kd) == list(range(m))
        # a micro-batch's backward follows its forward; W follows its B
        pos = {op: i for i, op in enumerate(ops)}
        for k in range(m):
            b = pos[("BW", k)] if schedule == "1f1b" else pos[("B", k)]
            assert pos[("F", k)] < b
            if schedule != "1f1b":
                assert b < pos[("W", k)]


def test_zbh1_defers_the_last_r_plus_1_weight_passes():
    pp, m = 4, 8
    for r in range(pp):
        ops = rank_ops("zbh1", pp, r, m)
        tail = ops[-(r + 1):]
        assert tail == [("W", k) for k in range(m - r - 1, m)]
        last_b = max(i for i, (kind, _) in enumerate(ops) if kind == "B")
        assert all(kind == "W" for kind, _ in ops[last_b + 1:])


def test_bubble_ordering_and_closed_forms():
    # unit costs: 1F1B bubble = (pp - 1)(F + B + W); the split backward sends earlier
    pp, m = 2, 8
    one = dict(F=[1.0] * pp, B=[1.0] * pp, W=[1.0] * pp)
    b = {s: simulate(s, pp, m, **one)["bubble"] for s in SCHEDULES}
    assert b["1f1b"] == pytest.approx(3.0)
    assert b["zb"] == pytest.approx(2.0)
    assert b["zbh1"] == pytest.approx(1.0)
    pp = 4
    one = dict(F=[1.0] * pp, B=[1.0] * pp, W=[1.0] * pp)
    b4 = {s: simulate(s, pp, m, **one)["bubble"] for s in SCHEDULES}
    assert b4["1f1b"] == pytest.approx((pp - 1) * 3.0)
    assert b4["zbh1"] < b4["zb"] < b4["1f1b"]


def test_zbh2_runs_ahead_and_reaches_the_startup_bound():
    """zbh2: rank r issues 2 (pp - r - 1) forwards before its first B and defers 2 (r + 1) W; at
    the measured BASELINE tp2pp2 per-micro-batch costs its bubble is the last stage's unavoidable
    first wait (stage 0's F + the hop), below zbh1's."""
    pp, m = 4, 8
    for r in range(pp):
        ops = rank_ops("zbh2", pp, r, m)
        first_b = min(i for i, (kind, _) in enumerate(ops) if kind == "B")
        assert first_b == 2 * (pp - r - 1) + 1          # the warm-up forwards, then the steady F
        n_def = min(m, 2 * (r + 1))
        assert ops[-n_def:] == [("W", k) for k in range(m - n_def, m)]
    F, B, W, hop = [9.10, 9.24], [11.68, 10.97], [4.77, 5.58], 0.52
    h1 = simulate("zbh1", 2, 8, F, B, W, p2p=hop)
    h2 = simulate("zbh2", 2, 8, F, B, W, p2p=hop)
    assert h2["bubble"] < h1["bubble"]
    assert h2["makespan"] == pytest.approx(F[0] + hop + 8 * (F[1] + B[1] + W[1]), abs=0.05)


def test_p2p_latency_and_uneven_stages():
    pp, m = 2, 8
    F, B, W = [1.0, 1.2], [1.0, 1.3], [0.8, 0.9]
    base = simulate("zbh1", pp, m, F, B, W)
    lat = simulate("zbh1", pp, m, F, B, W, p2p=0.25)
    assert lat["makespan"] > base["makespan"]
    # the heavier last stage bounds the step: makespan >= its busy time
    assert base["makespan"] >= m * (F[1] + B[1] + W[1]) - 1e-9
    assert base["bubble"] >= 0


def test_unknown_schedule_raises():
    with pytest.raises(ValueError):
        rank_ops("gpipe", 2, 0, 4)
