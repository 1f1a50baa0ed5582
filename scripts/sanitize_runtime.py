"""Run the host C++ runtime (``csrc/runtime/*.cpp``) under AddressSanitizer + UBSan.

SURVEY §5.2 asks for a sanitizer build target for the native extensions. GPU ASan / XNACK is not
available on the MI355X pool, so this covers the host side only: the GPT index builders
(``build_sample_idx`` in int32 and int64 mode, ``build_blending_indices``), the ZeRO-offload
``cpu_adam`` / ``cpu_sumsq`` (multi-threaded path included) and the fail-fast ``run_ranks``
supervisor. Every call is checked against a NumPy twin, so a sanitizer report OR a wrong answer
fails the run.

    python scripts/sanitize_runtime.py            # build (if stale) + run, exit 0 on success

The parent builds ``_runtime.so`` with ``-fsanitize=address,undefined`` into a scratch dir and
starts a CHILD interpreter with the sanitizer runtimes preloaded (no exec of the parent).
"""
from __future__ import annotations

import ctypes
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def _sample_idx_twin(sizes, doc_idx, seq_length, num_epochs, tokens_per_epoch):
    import numpy as np
    num_samples = (num_epochs * tokens_per_epoch - 1) // seq_length
    out = np.zeros((num_samples + 1, 2), dtype=np.int64)
    di, off = 0, 0
    for s in range(1, num_samples + 1):
        rem = seq_length + 1
        while rem != 0:
            dl = int(sizes[doc_idx[di]]) - off
            rem -= dl
            if rem <= 0:
                off += rem + dl - 1
                rem = 0
            else:
                di += 1
                off = 0
        out[s] = (di, off)
    return out


def _child(mod_dir):
    import numpy as np
    sys.path.insert(0, mod_dir)
    import _runtime as rt  # the sanitized build

    rng = np.random.RandomState(0)
    # --- build_sample_idx (int32 path) -------------------------------------------------------
    sizes = rng.randint(1, 300, size=500).astype(np.int32)
    doc_idx = np.concatenate([rng.permutation(500) for _ in range(3)]).astype(np.int32)
    tpe = int(sizes.sum())
    got = rt.build_sample_idx(sizes, doc_idx, 128, 3, tpe)
    assert got.dtype == np.int32, got.dtype
    np.testing.assert_array_equal(got.astype(np.int64), _sample_idx_twin(sizes, doc_idx, 128, 3, tpe))
    # int64 path: token count past INT32_MAX forces the wide template; keep the sample count tiny
    # by using a huge seq_length so the run stays small.
    big = np.full(4, 2**30, dtype=np.int32)
    bdoc = np.arange(4, dtype=np.int32)
    got64 = rt.build_sample_idx(big, bdoc, 2**30 - 1, 1, int(big.astype(np.int64).sum()))
    assert got64.dtype == np.int64, got64.dtype
    np.testing.assert_array_equal(got64, _sample_idx_twin(big, bdoc, 2**30 - 1, 1, int(big.astype(np.int64).sum())))
    # error paths must raise, not read out of bounds
    for bad in (dict(doc_idx=np.array([0, 9999], np.int32)), dict(doc_idx=np.array([0], np.int32))):
        try:
            rt.build_sample_idx(sizes[:2], bad["doc_idx"], 512, 4, 10_000)
        except (RuntimeError, ValueError):
            pass
        else:
            raise AssertionError("expected build_sample_idx to reject %r" % bad)

    # --- build_blending_indices --------------------------------------------------------------
    w = np.array([0.5, 0.3, 0.2])
    d, s = rt.build_blending_indices(w, 10_000)
    counts = np.bincount(d, minlength=3)
    assert np.all(np.abs(counts - w * 10_000) <= 1), counts
    for k in range(3):  # per-dataset sample indices are 0..count-1 in order
        np.testing.assert_array_equal(s[d == k], np.arange(counts[k]))

    # --- cpu_adam / cpu_sumsq (single- and multi-threaded) -----------------------------------
    for n in (1000, (1 << 18) + 7):
        p = rng.randn(n).astype(np.float32)
        g = rng.randn(n).astype(np.float32)
        m = np.zeros(n, np.float32)
        v = np.zeros(n, np.float32)
        out = np.zeros(n, np.uint16)
        p0 = p.copy()
        ptr = lambda a: a.ctypes.data_as(ctypes.c_void_p).value
        lr, b1, b2, eps, wd = 1e-3, 0.9, 0.999, 1e-8, 0.01
        rt.cpu_adam(ptr(p), ptr(g), ptr(m), ptr(v), ptr(out), n, lr, b1, b2, eps, wd, 1, True, 1.0, 4)
        m_ref = (1 - b1) * g
        v_ref = (1 - b2) * g * g
        p_ref = p0 * (1 - lr * wd) - lr * (m_ref / (1 - b1)) / (np.sqrt(v_ref / (1 - b2)) + eps)
        np.testing.assert_allclose(p, p_ref, rtol=1e-5, atol=1e-6)
        bf = (out.astype(np.uint32) << 16).view(np.float32)
        np.testing.assert_allclose(bf, p, rtol=1e-2, atol=1e-6)
        ss = rt.cpu_sumsq(ptr(g), n)
        assert abs(ss - float((g.astype(np.float64) ** 2).sum())) < 1e-6 * ss

    # --- run_ranks: success, and fail-fast on the first bad rank ------------------------------
    env = [f"{k}={v}" for k, v in os.environ.items() if not k.startswith("LD_PRELOAD")]
    job, status, first = rt.run_ranks([["/bin/true"], ["/bin/true"]], [env, env], grace=2.0)
    assert job == 0 and list(status) == [0, 0], (job, status)
    job, status, first = rt.run_ranks([["/bin/sh", "-c", "exit 3"], ["/bin/sleep", "30"]], [env, env], grace=1.0)
    assert job == 3 and first == 0, (job, status, first)
    print("[sanitize] runtime OK under ASan+UBSan: sample_idx(i32,i64), blending, cpu_adam, cpu_sumsq, run_ranks")


def main():
    if len(sys.argv) > 2 and sys.argv[1] == "--child":
        _child(sys.argv[2])
        return 0
    sys.path.insert(0, ROOT)
    from smdt_amd import _build
    out_dir = os.environ.get("SMDT_ASAN_DIR", "/tmp/smdt_runtime_asan")
    mod = _build.build_runtime_sanitized(out_dir, verbose="-v" in sys.argv)
    env = dict(os.environ)
    env["LD_PRELOAD"] = " ".join(_build.sanitizer_preload())
    # CPython's own allocations are reported as leaks at exit; every other check stays on.
    env["ASAN_OPTIONS"] = "detect_leaks=0:abort_on_error=0:halt_on_error=1"
    env["UBSAN_OPTIONS"] = "print_stacktrace=1:halt_on_error=1"
    r = subprocess.run([sys.executable, os.path.abspath(__file__), "--child", os.path.dirname(mod)], env=env)
    return r.returncode


if __name__ == "__main__":
    sys.exit(main())
