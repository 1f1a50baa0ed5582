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
    import smdt_amd.comm.smddp as S  # registers backend "smddp"
    dist.init_process_group(backend="smddp")
    t = torch.full((4,), float(rank + 1))
    dist.all_reduce(t)
    be = dist.get_backend()
    # the collectives a data-parallel script and the framework issue, all through the smddp group
    b = torch.full((3,), float(rank))
    dist.broadcast(b, src=1)
    gl = [torch.zeros(2) for _ in range(world)]
    dist.all_gather(gl, torch.full((2,), float(rank)))
    gt = torch.zeros(2 * world)
    dist.all_gather_into_tensor(gt, torch.full((2,), float(rank)))
    rs = torch.zeros(2)
    dist.reduce_scatter_tensor(rs, torch.arange(2.0 * world) + rank)
    objs = [None] * world
    dist.all_gather_object(objs, {"r": rank})
    dist.barrier()
    # unmodified torch DDP on the smddp group (the reference recipes' wrapping)
    torch.manual_seed(0)
    m = torch.nn.Linear(8, 4)
    ddp = S.DistributedDataParallel(m)      # torch DDP, buckets sized by comm/buckets.py
    x = torch.randn(6, 8, generator=torch.Generator().manual_seed(rank))
    ddp(x).square().sum().backward()
    g = m.weight.grad.clone()
    ref = [torch.zeros_like(g) for _ in range(world)]
    m2 = torch.nn.Linear(8, 4)
    m2.load_state_dict(m.state_dict())
    m2.zero_grad()
    m2(x).square().sum().backward()
    dist.all_gather(ref, m2.weight.grad)
    ok = torch.allclose(g, sum(ref) / world, atol=1e-5)
    stats = S.smddp_stats()
    dist.destroy_process_group()
    return t.tolist(), be, b.tolist(), [v.tolist() for v in gl], gt.tolist(), rs.tolist(), objs, ok, stats


@pytest.mark.slow
def test_smddp_backend_name_works_unmodified():
    """backend="smddp" (comm/smddp.SMDDPProcessGroup, a real c10d backend over RCCL / Gloo with the
    xGMI all-reduce path for GPU tensors): the collectives and torch DDP of the reference's DDP
    recipes run unchanged (CPU / Gloo here: every all-reduce takes the RCCL / Gloo path)."""
    outs = run_workers(_smddp_worker, 2)
    for r, (vals, be, b, gl, gt, rs, objs, ok, stats) in enumerate(outs):
        assert vals == [3.0] * 4 and be == "smddp"
        assert b == [1.0] * 3 and gl == [[0.0, 0.0], [1.0, 1.0]] and gt == [0.0, 0.0, 1.0, 1.0]
        assert rs == [4.0 * r + 1, 4.0 * r + 3]          # sum over ranks of (arange(4) + rank)[2r:2r+2]
        assert objs == [{"r": 0}, {"r": 1}] and ok
        assert stats["rccl_calls"] >= 2 and stats["xgmi_calls"] == 0


def test_host_runtime_under_asan_ubsan(tmp_path):
    """the native host runtime (index builders, cpu_adam, supervisor) built with
    -fsanitize=address,undefined and checked against NumPy twins (scripts/sanitize_runtime.py)."""
    env = dict(os.environ, SMDT_ASAN_DIR=str(tmp_path / "asan"))
    r = subprocess.run([sys.executable, os.path.join(HERE, "..", "scripts", "sanitize_runtime.py")],
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "runtime OK under ASan+UBSan" in r.stdout


def test_miopen_user_db_seeding(tmp_path, monkeypatch):
    """utils/miopen.seed_user_db: the shipped gfx950 find / perf databases (text) land in
    MIOPEN_USER_DB_PATH before the first convolution, and whatever MIOpen already wrote there is
    kept."""
    from smdt_amd.utils import miopen
    files = miopen.shipped_files()
    assert any(f.endswith(".ufdb.txt") for f in files) and any(f.endswith(".udb.txt") for f in files)
    target = tmp_path / "udb"
    target.mkdir()
    keep = target / files[0]
    keep.write_text("written by MIOpen\n")
    monkeypatch.setenv("MIOPEN_USER_DB_PATH", str(target))
    assert miopen.seed_user_db() == str(target)
    assert keep.read_text() == "written by MIOpen\n"
    for f in files[1:]:
        assert (target / f).read_bytes() == open(os.path.join(miopen._SHIPPED, f), "rb").read()
    # no MIOPEN_USER_DB_PATH: a per-user cache directory becomes it
    monkeypatch.delenv("MIOPEN_USER_DB_PATH")
    monkeypatch.setenv("HOME", str(tmp_path / "home"))
    d = miopen.seed_user_db()
    assert d == os.environ["MIOPEN_USER_DB_PATH"] and sorted(os.listdir(d)) == files
