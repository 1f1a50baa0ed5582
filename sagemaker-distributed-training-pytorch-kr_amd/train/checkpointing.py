"""Megatron-layout checkpoints.

Layout kept from the reference's Megatron recipe (`--save /opt/ml/model/`, "saving checkpoint at
iteration 2000", NB3:4582)::

    <save>/latest_checkpointed_iteration.txt          # "2000" (or "release")
    <save>/iter_0002000/mp_rank_TT[_PPP]/model_optim_rng.pt
    <save>/iter_0002000/mp_rank_TT[_PPP]/distrib_optim_dpDDD.pt   # ZeRO shards (one per DP rank)

Files hold only tensors and plain Python containers (args are stored as a primitive dict), so
they load with ``torch.load(..., weights_only=True)``. Writes go to a temp name and are renamed,
and the tracker file is written last by global rank 0 after a barrier, so a crash never leaves a
"latest" pointing at a half-written iteration. Flags honoured: ``--save``, ``--save-interval``,
``--load``, ``--no-save-optim``, ``--no-save-rng``, ``--no-load-optim``, ``--no-load-rng``,
``--finetune``, ``--exit-on-missing-checkpoint``, ``--use-checkpoint-args``
(/root/reference/3_training_megatron-lm/megatron/arguments.py:922-956).

``--async-save`` (Megatron-core's flag): the save only SNAPSHOTS the state — every device tensor
is copied on the current stream into pinned host memory (stream-ordered, so the next step's kernels
cannot change it) — and a writer thread serialises and renames the files while training goes on.
The step pays the device-to-host copy only (GPT-2 345M with Adam state: ~5.7 GB at ~25-50 GB/s)
instead of the serialisation and file writes (the reference logs 711.6 ms per save, NB3:4584).
The tracker is written once every rank's writer has finished: ``finalize_async_save`` is called
at the log interval (a MIN agreement over ranks, no wait) and before any exit or the next save
(blocking), so ``latest`` never points at an unfinished iteration.
"""
from __future__ import annotations

import os
import threading
import time
from typing import Optional

import torch
import torch.distributed as dist

from ..parallel import state as ps
from ..parallel.random import load_rng_state_dict, rng_state_dict

CHECKPOINT_VERSION = 3.0
TRACKER = "latest_checkpointed_iteration.txt"


def _rank0():
    return (not dist.is_initialized()) or dist.get_rank() == 0


def _barrier():
    if dist.is_initialized():
        dist.barrier()


def checkpoint_dir(root: str, iteration: int, release: bool = False) -> str:
    st = ps.get_state()
    d = "release" if release else f"iter_{iteration:07d}"
    sub = f"mp_rank_{st.tp_rank:02d}" if st.pp == 1 else f"mp_rank_{st.tp_rank:02d}_{st.pp_rank:03d}"
    return os.path.join(root, d, sub)


def _args_to_dict(args) -> dict:
    out = {}
    for k, v in vars(args).items():
        if isinstance(v, (int, float, str, bool)) or v is None:
            out[k] = v
        elif isinstance(v, (list, tuple)) and all(isinstance(x, (int, float, str, bool)) for x in v):
            out[k] = list(v)
        elif isinstance(v, torch.dtype):
            out[k] = str(v)
    return out


def _atomic_save(obj, path):
    os.makedirs(os.path.dirname(path), exist_ok=True)
    tmp = f"{path}.tmp{os.getpid()}"
    torch.save(obj, tmp)
    os.replace(tmp, path)


def _unwrap(model):
    return model.module if hasattr(model, "module") else model


_PENDING = {"thread": None, "iteration": None, "save_dir": None, "error": None}


def _snapshot(obj, copies):
    """``obj`` with every tensor replaced by a host copy (device tensors: pinned, non-blocking on
    the current stream; ``copies`` collects them so one event can cover all)."""
    if isinstance(obj, torch.Tensor):
        t = obj.detach()
        if t.is_cuda:
            h = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
            h.copy_(t, non_blocking=True)
            copies.append(h)
            return h
        return t.clone()
    if isinstance(obj, dict):
        return type(obj)((k, _snapshot(v, copies)) for k, v in obj.items())
    if isinstance(obj, tuple) and hasattr(obj, "_fields"):   # namedtuple
        return type(obj)(*(_snapshot(v, copies) for v in obj))
    if isinstance(obj, (list, tuple)):
        return type(obj)(_snapshot(v, copies) for v in obj)
    return obj


def _writer(jobs, event):
    try:
        if event is not None:
            event.synchronize()
        for obj, path in jobs:
            _atomic_save(obj, path)
    except Exception as e:  # noqa: BLE001 - reported by finalize_async_save
        _PENDING["error"] = e


def _all_ranks(flag: bool) -> bool:
    if not dist.is_initialized():
        return flag
    t = torch.tensor([int(flag)])
    if torch.cuda.is_available() and dist.get_backend() in ("nccl", "smddp"):
        t = t.cuda()
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return bool(t.item())


def finalize_async_save(blocking: bool = True) -> bool:
    """Collective. Completes a pending ``--async-save``: once every rank's writer thread is done,
    global rank 0 writes the tracker. ``blocking=False`` only checks (returns False while a writer
    is still running somewhere). Every rank must call it at the same points."""
    th = _PENDING["thread"]
    if th is None:            # the same on every rank: saves start collectively
        return True
    if blocking:
        th.join()
    if not _all_ranks(not th.is_alive()):
        return False
    ok = _all_ranks(_PENDING["error"] is None)
    err = _PENDING["error"]
    it, save_dir = _PENDING["iteration"], _PENDING["save_dir"]
    _PENDING.update(thread=None, iteration=None, save_dir=None, error=None)
    if not ok:
        raise RuntimeError(f"async checkpoint write of iteration {it} failed"
                           + (f" on this rank: {err}" if err is not None else " on another rank"))
    _barrier()
    if _rank0():
        with open(os.path.join(save_dir, TRACKER), "w") as f:
            f.write(str(it))
        print(f"  successfully saved checkpoint at iteration {it:7d} to {save_dir} (async)", flush=True)
    _barrier()
    return True


def save_checkpoint(iteration: int, model, optimizer=None, scheduler=None, args=None, save_dir: Optional[str] = None,
                    extra: Optional[dict] = None, async_save: Optional[bool] = None):
    save_dir = save_dir or args.save
    if async_save is None:
        async_save = bool(getattr(args, "async_save", False)) if args is not None else False
    finalize_async_save(blocking=True)   # one save in flight at a time
    t0 = time.time()
    jobs = []
    if hasattr(model, "wait_param_gather"):  # overlapped ZeRO all-gather still in flight
        model.wait_param_gather()
    if _rank0():
        print(f"saving checkpoint at iteration {iteration:7d} to {save_dir}", flush=True)
    st = ps.get_state()
    d = checkpoint_dir(save_dir, iteration)
    no_optim = bool(getattr(args, "no_save_optim", False)) if args is not None else False
    no_rng = bool(getattr(args, "no_save_rng", False)) if args is not None else False
    zero = optimizer is not None and getattr(optimizer, "zero", False)
    if st.dp_rank == 0 and st.cp_rank == 0:
        sd = {"checkpoint_version": CHECKPOINT_VERSION, "iteration": iteration,
              "model": _unwrap(model).state_dict()}
        if args is not None:
            sd["args"] = _args_to_dict(args)
        if optimizer is not None and not no_optim and not zero:
            sd["optimizer"] = optimizer.state_dict()
        if scheduler is not None and not no_optim:
            sd["opt_param_scheduler"] = scheduler.state_dict()
        if not no_rng:
            sd["rng_state"] = _rng_for_save()
        if extra:
            sd.update(extra)
        jobs.append((sd, os.path.join(d, "model_optim_rng.pt")))
    if st.cp > 1 and st.dp_rank == 0 and st.cp_rank > 0 and not no_rng:
        # Context-parallel ranks run shifted Philox streams (parallel/random.py): each keeps its own
        # so a resumed run draws the same dropout masks as one that never stopped.
        jobs.append(({"iteration": iteration, "rng_state": _rng_for_save()},
                     os.path.join(d, f"rng_cp{st.cp_rank:03d}.pt")))
    if zero and not no_optim:
        jobs.append(({"iteration": iteration, "optimizer": optimizer.state_dict()},
                     os.path.join(d, f"distrib_optim_dp{st.dp_cp_rank:03d}.pt")))
    if async_save:
        copies = []
        snap = [(_snapshot(obj, copies), path) for obj, path in jobs]
        ev = None
        if copies and torch.cuda.is_available():
            ev = torch.cuda.Event()
            ev.record()
        th = threading.Thread(target=_writer, args=(snap, ev), name=f"smdt-ckpt-{iteration}", daemon=False)
        _PENDING.update(thread=th, iteration=iteration, save_dir=save_dir, error=None)
        th.start()
        return time.time() - t0
    for obj, path in jobs:
        _atomic_save(obj, path)
    _barrier()
    if _rank0():
        with open(os.path.join(save_dir, TRACKER), "w") as f:
            f.write(str(iteration))
        print(f"  successfully saved checkpoint at iteration {iteration:7d} to {save_dir}", flush=True)
    _barrier()
    return time.time() - t0


def _rng_for_save():
    r = rng_state_dict()
    # numpy / python states are tuples with non-tensor payloads: keep the tensor-able parts only
    out = {k: v for k, v in r.items() if k in ("default", "tp", "torch_cpu", "torch_cuda")}
    np_state = r.get("numpy")
    if np_state is not None:
        out["numpy_keys"] = torch.from_numpy(np_state[1].astype("int64"))
        out["numpy_pos"] = int(np_state[2])
    return out


def read_tracker(load_dir: str):
    p = os.path.join(load_dir, TRACKER)
    if not os.path.isfile(p):
        return None, False
    s = open(p).read().strip()
    if s == "release":
        return 0, True
    return int(s), False


# The model-shape arguments ``--use-checkpoint-args`` takes from the checkpoint (Megatron's
# load_args_from_checkpoint, /root/reference/3_training_megatron-lm/megatron/checkpointing.py).
CHECKPOINT_ARGS = ("num_layers", "hidden_size", "ffn_hidden_size", "seq_length", "num_attention_heads",
                   "num_query_groups", "group_query_attention", "kv_channels", "max_position_embeddings",
                   "position_embedding_type", "add_position_embedding", "use_rotary_position_embeddings",
                   "rotary_percent", "add_bias_linear", "swiglu", "untie_embeddings_and_output_weights",
                   "normalization", "layernorm_epsilon", "tokenizer_type", "vocab_size", "padded_vocab_size",
                   "make_vocab_size_divisible_by", "tensor_model_parallel_size",
                   "pipeline_model_parallel_size")


def load_args_from_checkpoint(args, load_dir: Optional[str] = None) -> bool:
    """``--use-checkpoint-args``: overwrite the model-shape arguments with the ones the checkpoint
    under ``--load`` was saved with (before ``validate_args``). Reads the tensor/pipeline rank-0
    file only, with ``weights_only=True``. Returns False (args untouched) when there is none."""
    load_dir = load_dir or getattr(args, "load", None)
    if not load_dir:
        raise SystemExit("--use-checkpoint-args needs --load")
    it, release = read_tracker(load_dir)
    if it is None:
        print(f"WARNING: --use-checkpoint-args: no checkpoint under {load_dir}; using the command line",
              flush=True)
        return False
    d = os.path.join(load_dir, "release" if release else f"iter_{it:07d}")
    for sub in ("mp_rank_00", "mp_rank_00_000"):
        f = os.path.join(d, sub, "model_optim_rng.pt")
        if os.path.isfile(f):
            break
    else:
        raise SystemExit(f"--use-checkpoint-args: no rank-0 checkpoint file under {d}")
    saved = torch.load(f, map_location="cpu", weights_only=True).get("args", {})
    for k in CHECKPOINT_ARGS:
        if k in saved and hasattr(args, k):
            setattr(args, k, saved[k])
    return True


def load_checkpoint(model, optimizer=None, scheduler=None, args=None, load_dir: Optional[str] = None,
                    strict: bool = True) -> int:
    """Returns the iteration to resume from (0 when nothing was loaded)."""
    load_dir = load_dir or (args.load if args is not None else None)
    if not load_dir:
        return 0
    it, release = read_tracker(load_dir)
    if it is None:
        if args is not None and getattr(args, "exit_on_missing_checkpoint", False):
            raise SystemExit(f"--exit-on-missing-checkpoint: no checkpoint under {load_dir}")
        if _rank0():
            print(f"WARNING: could not find the metadata file {os.path.join(load_dir, TRACKER)}; "
                  "training from random initialization", flush=True)
        return 0
    d = checkpoint_dir(load_dir, it, release)
    sd = torch.load(os.path.join(d, "model_optim_rng.pt"), map_location="cpu", weights_only=True)
    _unwrap(model).load_state_dict(sd["model"], strict=strict)
    finetune = bool(getattr(args, "finetune", False)) if args is not None else False
    no_load_optim = bool(getattr(args, "no_load_optim", False)) if args is not None else False
    no_load_rng = bool(getattr(args, "no_load_rng", False)) if args is not None else False
    optim_loaded = False
    if optimizer is not None and not (finetune or no_load_optim or release):
        if getattr(optimizer, "zero", False):
            st = ps.get_state()
            p = os.path.join(d, f"distrib_optim_dp{st.dp_cp_rank:03d}.pt")
            if os.path.isfile(p):
                optimizer.load_state_dict(torch.load(p, map_location="cpu", weights_only=True)["optimizer"])
                optim_loaded = True
            elif not bool(getattr(args, "no_save_optim", False)):
                # a ZeRO checkpoint whose shard for this DP rank is missing cannot resume the
                # optimizer: say so (the masters are refreshed from the loaded weights below)
                print(f"WARNING: rank {dist.get_rank() if dist.is_initialized() else 0}: ZeRO optimizer shard "
                      f"{p} not found; optimizer state restarts from the loaded weights", flush=True)
        elif "optimizer" in sd:
            optimizer.load_state_dict(sd["optimizer"])
            optim_loaded = True
        if scheduler is not None and "opt_param_scheduler" in sd:
            scheduler.load_state_dict(sd["opt_param_scheduler"])
    if optimizer is not None and not optim_loaded:
        # The optimizer was built before the load, so its fp32 masters still hold the random-init
        # weights: refresh them from the loaded model, or the first step writes them back.
        sync = getattr(optimizer, "reload_model_params", None)
        if sync is not None:
            sync()
    st = ps.get_state()
    rng_src = sd
    if st.cp > 1 and st.cp_rank > 0:
        p = os.path.join(d, f"rng_cp{st.cp_rank:03d}.pt")
        rng_src = torch.load(p, map_location="cpu", weights_only=True) if os.path.isfile(p) else {}
    if "rng_state" in rng_src and not (finetune or no_load_rng or release):
        r = dict(rng_src["rng_state"])
        rs = {k: v for k, v in r.items() if k in ("default", "tp", "torch_cpu", "torch_cuda")}
        if "numpy_keys" in r:  # data-side randomness (shuffles, augmentation) resumes too
            import numpy as np
            rs["numpy"] = ("MT19937", r["numpy_keys"].numpy().astype(np.uint32), int(r["numpy_pos"]), 0, 0.0)
        load_rng_state_dict(rs)
    if args is not None and "args" in sd:
        for k in ("consumed_train_samples", "consumed_valid_samples"):
            if k in sd["args"]:
                setattr(args, k, sd["args"][k])
    _barrier()
    if _rank0():
        print(f"  successfully loaded checkpoint from {load_dir} at iteration {it}", flush=True)
    return 0 if (finetune or release) else it
