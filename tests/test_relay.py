"""Multi-path TP-pair exchange over xGMI (comm/relay.py, csrc/kernels/xgmi_relay.hip).

GPU tests run the exact kernel and protocol on one MI355X: W virtual ranks in one launch
(loopback: every "peer" buffer is local HBM, so this checks routing, slot parities and the
slot-reuse handshake, not link speed) and 4 real processes on cuda:0 exchanging through HIP-IPC
mappings (the cross-process path, incl. the tensor-parallel ring integration). The numbers that
decide whether training uses the relay come from ``XgmiRelay.tune`` on the real node.
"""
import os
import pickle
import tempfile

import pytest
import torch

from smdt_amd.comm import relay


def test_mode_parsing(monkeypatch):
    monkeypatch.delenv("SMDT_TP_RELAY", raising=False)
    assert relay.mode() == "auto"
    for v, m in (("0", "off"), ("off", "off"), ("1", "on"), ("ON", "on"), ("auto", "auto")):
        monkeypatch.setenv("SMDT_TP_RELAY", v)
        assert relay.mode() == m


def test_not_applicable_without_gpu_group():
    # no process group / no GPU: nothing is built and the TP ring keeps RCCL
    assert relay.create_for_pairs(None) is None
    assert relay.engine_for(None) is None


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 4, 8])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_loopback_exchange(world, dtype):
    """Row r of the output is row r ^ 1 of the input, over 6 consecutive calls (both slot parities
    and the freed-slot wait), for sizes that fill every part, leave the last part short, and leave
    some parts empty."""
    torch.manual_seed(world)
    lb = relay.XgmiRelayLoopback(world, slot_bytes=1 << 20, sub=2)
    try:
        es = torch.tensor([], dtype=dtype).element_size()
        cap = world * lb.slot // 2 // es
        for n in (16 // es, 1000 * 16 // es, cap // 3 // 8 * 8, cap):
            for rep in range(6):
                x = torch.randn(world, n, device="cuda").to(dtype)
                y = lb.exchange(x)
                torch.cuda.synchronize()
                perm = torch.tensor([r ^ 1 for r in range(world)], device="cuda")
                assert torch.equal(y, x[perm]), (n, rep)
        assert lb.errors() == [0] * world
    finally:
        lb.close()


@pytest.mark.gpu
def test_loopback_rejects_oversized_call():
    lb = relay.XgmiRelayLoopback(4, slot_bytes=1 << 20, sub=2)
    try:
        n = 4 * lb.slot // 2 // 4 + 64
        with pytest.raises(RuntimeError):
            lb.exchange(torch.zeros(4, n, device="cuda"))
    finally:
        lb.close()


@pytest.mark.gpu
def test_cross_process_relay_and_tp_ring():
    """4 processes on cuda:0, pairs (0,1) (2,3): HIP-IPC handle exchange, the engine's own
    validation against p2p, chunked messages, the async handle, and ag_ring / rs_ring of the
    tensor-parallel layers routed through the relay."""
    import torch.multiprocessing as mp

    import dist_workers as W
    from _dist import free_port

    world = 4
    port = free_port()
    with tempfile.TemporaryDirectory() as d:
        ctx = mp.get_context("spawn")
        procs = [ctx.Process(target=W.relay_ipc_worker, args=(r, world, port, d)) for r in range(world)]
        for p in procs:
            p.start()
        for p in procs:
            p.join(120)
        for p in procs:
            if p.is_alive():
                p.kill()
        out = []
        for r in range(world):
            path = os.path.join(d, f"r{r}.pkl")
            assert os.path.exists(path), f"rank {r} wrote no result (exit {procs[r].exitcode})"
            with open(path, "rb") as f:  # written by this test's own workers
                out.append(pickle.load(f))
    for r, res in enumerate(out):
        assert res["err"] is None, f"rank {r}:\n{res['err']}"
        assert res["error_word"] == 0 and all(res["ok"]) and len(res["ok"]) == 10, (r, res)


@pytest.mark.gpu
def test_tensor_parallel_mlp_over_relay_matches_fp32_reference():
    """Sequence-parallel TP=2 MLP (column fc1 + bias + GeLU, row fc2) in 4 processes on one GPU with
    every ring exchange on the relay kernel: outputs and all gradient shards match an fp32
    reference of the full MLP, over two iterations."""
    import torch.multiprocessing as mp

    import dist_workers as W
    from _dist import free_port

    world = 4
    port = free_port()
    with tempfile.TemporaryDirectory() as d:
        ctx = mp.get_context("spawn")
        procs = [ctx.Process(target=W.relay_tp_mlp_worker, args=(r, world, port, d)) for r in range(world)]
        for p in procs:
            p.start()
        for p in procs:
            p.join(120)
        for p in procs:
            if p.is_alive():
                p.kill()
        out = []
        for r in range(world):
            path = os.path.join(d, f"r{r}.pkl")
            assert os.path.exists(path), f"rank {r} wrote no result (exit {procs[r].exitcode})"
            with open(path, "rb") as f:  # written by this test's own workers
                out.append(pickle.load(f))
    for r, res in enumerate(out):
        assert res["err"] is None, f"rank {r}:\n{res['err']}"
        assert res["error_word"] == 0 and res["calls"] >= 8, (r, res)
        bad = {k: v for k, v in res["rel"].items() if not v < 2e-2}
        assert not bad, (r, bad)


@pytest.mark.gpu
def test_relay_exchange_replays_from_a_hip_graph():
    """2 processes on cuda:0 (one TP pair) capture the relay exchange in a HIP
    graph and replay it 20x with fresh inputs, eager exchanges in between; every replay equals the
    partner's input bit for bit. Possible because the relay's epochs are device counters, bumped
    in-stream, not host values baked into the captured launches."""
    import torch.multiprocessing as mp

    import dist_workers as W
    from _dist import free_port

    world = 2
    port = free_port()
    with tempfile.TemporaryDirectory() as d:
        ctx = mp.get_context("spawn")
        procs = [ctx.Process(target=W.relay_graph_worker, args=(r, world, port, d)) for r in range(world)]
        for p in procs:
            p.start()
        for p in procs:
            p.join(120)
        for p in procs:
            if p.is_alive():
                p.kill()
        out = []
        for r in range(world):
            path = os.path.join(d, f"r{r}.pkl")
            assert os.path.exists(path), f"rank {r} wrote no result (exit {procs[r].exitcode})"
            with open(path, "rb") as f:  # written by this test's own workers
                out.append(pickle.load(f))
    for r, res in enumerate(out):
        assert res["err"] is None, f"rank {r}:\n{res['err']}"
        assert res["error_word"] == 0 and res["replays"] == 20 and all(res["ok"]) and len(res["ok"]) == 27, (r, res)
