"""benchmarks/convergence.py on CPU: the Markov corpus is deterministic and obeys its successor
table (so ln 4 is the achievable loss), and the comparison table reads the two loss curves."""
import json
import math
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "benchmarks"))
import convergence as C  # noqa: E402


def test_markov_corpus_is_deterministic_and_follows_its_table():
    a = C.markov_batches(3, 2, 64, states=32, fanout=4, seed=3)
    b = C.markov_batches(3, 2, 64, states=32, fanout=4, seed=3)
    assert a.shape == (3, 2, 65) and np.array_equal(a, b)
    succ = np.random.default_rng(3).integers(0, 32, size=(32, 4))
    flat = a.reshape(-1, 65)
    for row in flat:
        for t in range(64):
            assert row[t + 1] in succ[row[t]]


def test_compare_table(tmp_path):
    k1 = [10.0 - 0.01 * i for i in range(200)]
    k0 = [x + 0.002 for x in k1]
    p1, p0 = tmp_path / "k1.json", tmp_path / "k0.json"
    p1.write_text(json.dumps({"losses": k1}))
    p0.write_text(json.dumps({"losses": k0}))
    md = C.compare(str(p1), str(p0), label0="control")
    assert "| quantity | HIP kernels | control |" in md
    assert "max |difference| over all 200 steps: 0.0020" in md
    assert f"{math.log(4):.4f}" in md
