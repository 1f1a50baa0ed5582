"""benchmarks/predict_scaling.py's tables from synthetic per-stage measurements (CPU): the
schedule rows are ordered as the simulator says (zbh1 <= zb <= 1f1b bubble) and the GPT-3 TP4
rows charge the one-link ring more than the three-link exchange, and the direct exchange's row
pieces (simulated per exchange against its own GEMMs) less than whole chunks; the GPT-2 N = 8
TP-pair exchanges, simulated the same way, cost more over one link than over the relay."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _rec(ms, f=None, tok=65536):
    return {"ms_per_step": ms, "phase_ms": None, "tokens_per_step": tok, "args": [],
            "fbw_ms": None if f is None else {"F": f[0], "B": f[1], "W": f[2], "micro_batches": 8}}


def test_prediction_tables(tmp_path):
    m = {"n1_dp": _rec(160.0), "tp2pp2_stage0": _rec(175.0, (6.0, 8.0, 6.5)),
         "tp2pp2_stage1": _rec(178.0, (7.0, 8.5, 6.0)), "tp2pp2_stage1_even": _rec(185.0, (7.5, 9.0, 6.3)),
         "gpt3_tp4_stage0": _rec(370.0, (13.0, 18.0, 14.0), tok=65536),
         "gpt3_tp4_stage1": _rec(385.0, (14.0, 19.0, 14.0), tok=65536), "gpt3_n1": _rec(330.0, tok=8192)}
    src = tmp_path / "m.json"
    src.write_text(json.dumps({"measured": m}))
    r = subprocess.run([sys.executable, os.path.join(ROOT, "benchmarks", "predict_scaling.py"), "--from-json", str(src),
                        "--out", str(tmp_path)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads((tmp_path / "predicted.json").read_text())
    n8 = {row["layout"].split(", ")[-1]: row for row in out["rows"] if row["N"] == 8}
    assert n8["zbh2"]["bubble_ms"] <= n8["zbh1"]["bubble_ms"] <= n8["zb"]["bubble_ms"] <= n8["1f1b"]["bubble_ms"]
    assert n8["zbh1"]["efficiency_vs_n1"] > n8["1f1b"]["efficiency_vs_n1"]
    assert "interleaved vpp2 (even 12|12 split)" in n8
    # the TP-pair exchanges simulated per exchange: the relay (4 links' worth) exposes less than
    # RCCL's single link, and both more than the assumed-hidden zbh2 row
    rl = n8["TP exchange relay"]
    one = n8["TP exchange RCCL p2p"]
    assert n8["zbh2"]["predicted_ms"] < rl["predicted_ms"] < one["predicted_ms"]
    assert rl["bubble_ms"] == n8["zbh2"]["bubble_ms"]
    g3 = out["gpt3_rows"]
    assert len(g3) == 4
    ex = [row["exposed_comm_ms"] for row in g3]   # ring, direct whole chunks, 2 pieces, 4 pieces
    assert ex[0] > ex[1] > ex[2] > ex[3] > 0
    assert all(0 < row["efficiency_vs_n1"] < 1.5 for row in g3)
    assert (tmp_path / "predicted.md").read_text().count("\n") >= 10
