"""Failure detection / fault injection / collective-sequence checking."""
import os
import subprocess
import sys
import time

import pytest
import torch

from smdt_amd.utils.debug import parse_fault_spec

from _dist import free_port, run_workers

HERE = os.path.dirname(os.path.abspath(__file__))


def test_parse_fault_spec():
    f = parse_fault_spec("rank=1, step=3, mode=hang")
    assert f == {"rank": 1, "step": 3, "mode": "hang"}
    assert parse_fault_spec("mode=nan")["rank"] is None


def _tracer_worker(rank, world):
    import torch.distributed as dist
    from smdt_amd.utils.debug import CollectiveTracer
    dist.init_process_group("gloo")
    solo = [dist.new_group([r]) for r in range(world)]  # singleton groups: complete locally
    tr = CollectiveTracer().install()
    x = torch.ones(8)
    dist.all_reduce(x)
    ok = tr.check()
    # rank 1 issues one extra collective (on its own singleton group, so nothing blocks):
    # the per-rank sequences now disagree, which is what would hang a real job
    if rank == 1:
        dist.all_reduce(torch.ones(3), group=solo[1])
    bad = tr.check()
    tr.uninstall()
    dist.destroy_process_group()
    return ok, bad


@pytest.mark.slow
def test_collective_tracer_flags_divergent_rank():
    outs = run_workers(_tracer_worker, 2)
    for ok, bad in outs:
        assert ok is None
        assert bad is not None and "disagree" in bad and "rank 1" in bad


def _supervise(extra_env, args=(), grace=5, max_run=120):
    from smdt_amd import _runtime
    port = free_port()
    argvs, envs = [], []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE="2", LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), **extra_env)
        argvs.append([sys.executable, os.path.join(HERE, "_fault_worker.py"), *args])
        envs.append([f"{k}={v}" for k, v in env.items()])
    t0 = time.time()
    status, per, first = _runtime.run_ranks(argvs, envs, grace, max_run)
    return status, per, first, time.time() - t0


@pytest.mark.slow
def test_injected_rank_exit_fails_job_fast():
    """rank 1 dies at step 3 while rank 0 waits in an all-reduce: the supervisor must propagate
    rank 1's status and kill rank 0 right away (not after the 120 s collective timeout)."""
    status, per, first, dt = _supervise({"SMDT_FAULT_INJECT": "rank=1,step=3,mode=exit"})
    assert first == 1 and per[1] == 13 and status == 13, (status, per, first)
    assert dt < 60, dt


@pytest.mark.slow
def test_clean_job_succeeds_under_supervisor():
    status, per, first, _ = _supervise({})
    assert status == 0 and per == [0, 0] and first == -1


def test_step_watchdog_dumps_stacks_and_aborts():
    p = subprocess.run([sys.executable, os.path.join(HERE, "_fault_worker.py"), "watchdog"], capture_output=True,
                       text=True, timeout=60)
    assert p.returncode == -6, p.returncode
    assert "step exceeded" in p.stderr and "_fault_worker.py" in p.stderr


def _smddp_worker(rank, world):
    import torch.distributed as dist
    import smdt_amd.comm.smddp  # noqa: F401  (registers backend "smddp")
    dist.init_process_group(backend="smddp")
    t = torch.full((4,), float(rank + 1))
    dist.all_reduce(t)
    be = dist.get_backend()
    dist.destroy_process_group()
    return t.tolist(), be


@pytest.mark.slow
def test_smddp_backend_name_works_unmodified():
    outs = run_workers(_smddp_worker, 2)
    for vals, be in outs:
        assert vals == [3.0] * 4 and be == "smddp"


def test_host_runtime_under_asan_ubsan(tmp_path):
    """the native host runtime (index builders, cpu_adam, supervisor) built with
    -fsanitize=address,undefined and checked against NumPy twins (scripts/sanitize_runtime.py)."""
    env = dict(os.environ, SMDT_ASAN_DIR=str(tmp_path / "asan"))
    r = subprocess.run([sys.executable, os.path.join(HERE, "..", "scripts", "sanitize_runtime.py")],
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "runtime OK under ASan+UBSan" in r.stdout
