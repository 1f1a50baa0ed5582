"""Multi-process test harness on CPU/gloo (the analogue of the reference's local mode)."""
import os
import pickle
import socket
import tempfile
import traceback

import torch.multiprocessing as mp


_NEXT = [0]


def free_port():
    """A free port BELOW the kernel's ephemeral range (32768+), in a block of its own per xdist
    worker: an ephemeral port probed free here could be taken by another test's Gloo connection
    before rank 0's store binds it (a parallel run then hung in rendezvous)."""
    w = os.environ.get("PYTEST_XDIST_WORKER", "gw0")
    wid = int(w[2:]) if w[2:].isdigit() else 0
    base = 10000 + (wid % 16) * 1000
    for _ in range(1000):
        port = base + (os.getpid() * 7 + _NEXT[0]) % 1000
        _NEXT[0] += 1
        with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
            try:
                s.bind(("127.0.0.1", port))
            except OSError:
                continue
            return port
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _entry(rank, world, port, fn, args, outdir, use_ompi):
    env = {"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)}
    if use_ompi:
        env.update({"OMPI_COMM_WORLD_RANK": str(rank), "OMPI_COMM_WORLD_SIZE": str(world),
                    "OMPI_COMM_WORLD_LOCAL_RANK": str(rank)})
        for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
            os.environ.pop(k, None)
    else:
        env.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank)})
    os.environ.update(env)
    os.environ["CUDA_VISIBLE_DEVICES"] = ""
    try:
        res = fn(rank, world, *args)
        err = None
    except Exception:  # pragma: no cover - reported by the parent
        res, err = None, traceback.format_exc()
    with open(os.path.join(outdir, f"r{rank}.pkl"), "wb") as f:
        pickle.dump((res, err), f)


def run_workers(fn, world, *args, use_ompi=False, timeout=300):
    """Run ``fn(rank, world, *args)`` in ``world`` spawned processes; return per-rank results."""
    port = free_port()
    with tempfile.TemporaryDirectory() as d:
        ctx = mp.get_context("spawn")
        procs = [ctx.Process(target=_entry, args=(r, world, port, fn, args, d, use_ompi)) for r in range(world)]
        for p in procs:
            p.start()
        for p in procs:
            p.join(timeout)
        for p in procs:
            if p.is_alive():
                p.kill()
                raise RuntimeError("worker timed out")
        out = []
        for r in range(world):
            path = os.path.join(d, f"r{r}.pkl")
            if not os.path.exists(path):
                raise RuntimeError(f"rank {r} produced no result (exit code {procs[r].exitcode})")
            with open(path, "rb") as f:  # written by our own workers in this test run
                res, err = pickle.load(f)
            if err:
                raise RuntimeError(f"rank {r} failed:\n{err}")
            out.append(res)
        return out
