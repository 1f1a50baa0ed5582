"""ZeRO engine driven by a DeepSpeed JSON config.

The reference hands ``--deepspeed configs/default_offload_opt_param.json`` to the HF Trainer,
which resolves every ``"auto"`` from the TrainingArguments and calls ``deepspeed.initialize``
(/root/reference/4_training_alpaca_deepspeed/configs/default_offload_opt_param.json:1-48,
train.py:243-244). This module is the MI355X-native equivalent:

* ``resolve_ds_config``  — HF's "auto" rules (micro batch, GA, global batch, clipping, AdamW
  lr/betas/eps/wd, WarmupDecayLR min/max/warmup/total, reduce/prefetch/persistence sizes from the
  hidden size) + consistency checks for explicit values;
* ``ZeroEngine``         — stage 0: bucketed all-reduce; stage 1: bucketed grad reduce-scatter
  overlapped with backward into a full flat fp32 buffer, fused AdamW HIP kernel on this rank's
  fp32 shard (master + moments), bf16 param all-gather; stage 2: the same with the gradients
  themselves partitioned — a bucket's fp32 buffer lives only while it accumulates, the persistent
  gradient storage is this rank's shard (parallel/distributed.py, ``zero_stage``); stage 3: the
  bf16 parameters partitioned too, gathered per transformer layer with traced prefetch and
  released after use (parallel/zero3.py), ``stage3_prefetch_bucket_size`` /
  ``stage3_param_persistence_threshold`` honoured, and ``offload_param: cpu`` keeping the shards in
  pinned host memory (H2D before each gather). Optimizer offload to CPU
  (``offload_optimizer.device == "cpu"``) runs AdamW on the host with the native multithreaded
  kernel in ``_runtime`` (DeepSpeed's cpu_adam equivalent);
* checkpoints in DeepSpeed's layout (``global_stepN/mp_rank_00_model_states.pt``,
  ``{bf16_,}zero_pp_rank_R_mp_rank_00_optim_states.pt``, ``latest``) and ``zero_to_fp32``
  consolidation.
"""
from __future__ import annotations

import json
import math
import os
import warnings
from contextlib import nullcontext
from typing import Dict, Optional

import torch
import torch.distributed as dist

from ..optim.lr_scheduler import LambdaWarmupScheduler, WarmupDecayLR
from ..optim.optimizer import ConstantLossScaler, DynamicLossScaler, MixedPrecisionAdam
from ..parallel import state as ps
from ..parallel.distributed import DistributedDataParallel

AUTO = "auto"
MIN_BUCKET = 16 * 1024 * 1024  # elements; xGMI rings want few, large collectives


def _is_auto(v):
    return isinstance(v, str) and v == AUTO


def load_ds_config(cfg) -> Dict:
    if cfg is None:
        return {}
    if isinstance(cfg, dict):
        return json.loads(json.dumps(cfg))
    with open(cfg) as f:
        return json.load(f)


def resolve_ds_config(cfg: Dict, args, hidden_size: int, world_size: int, num_training_steps: int) -> Dict:
    """Fill ``"auto"`` like ``transformers.integrations.deepspeed.HfTrainerDeepSpeedConfig``."""
    cfg = json.loads(json.dumps(cfg))
    mismatches = []

    def fill(d, key, value, name):
        if key not in d:
            return
        if _is_auto(d[key]):
            d[key] = value
        elif d[key] != value and value is not None:
            mismatches.append(f"- ds {key}={d[key]} vs hf {name}={value}")

    mbs, ga = args.per_device_train_batch_size, args.gradient_accumulation_steps
    fill(cfg, "train_micro_batch_size_per_gpu", mbs, "per_device_train_batch_size")
    fill(cfg, "gradient_accumulation_steps", ga, "gradient_accumulation_steps")
    fill(cfg, "train_batch_size", mbs * ga * world_size, "train_batch_size (calculated)")
    fill(cfg, "gradient_clipping", args.max_grad_norm, "max_grad_norm")
    opt = cfg.get("optimizer", {}).get("params", {})
    fill(opt, "lr", args.learning_rate, "learning_rate")
    fill(opt, "betas", [args.adam_beta1, args.adam_beta2], "adam_beta1+adam_beta2")
    fill(opt, "eps", args.adam_epsilon, "adam_epsilon")
    fill(opt, "weight_decay", args.weight_decay, "weight_decay")
    sch = cfg.get("scheduler", {}).get("params", {})
    fill(sch, "warmup_min_lr", 0, "warmup_min_lr")
    fill(sch, "warmup_max_lr", args.learning_rate, "learning_rate")
    fill(sch, "warmup_num_steps", args.get_warmup_steps(num_training_steps), "warmup_steps")
    fill(sch, "total_num_steps", num_training_steps, "max_steps")
    for k in ("fp16", "bf16"):
        if k in cfg and _is_auto(cfg[k].get("enabled")):
            cfg[k]["enabled"] = bool(getattr(args, k))
    z = cfg.get("zero_optimization", {})
    for key, val in (("reduce_bucket_size", hidden_size * hidden_size),
                     ("stage3_prefetch_bucket_size", int(0.9 * hidden_size * hidden_size)),
                     ("stage3_param_persistence_threshold", 10 * hidden_size)):
        if _is_auto(z.get(key)):
            z[key] = val
    if mismatches:
        raise ValueError("DeepSpeed config values differ from the TrainingArguments:\n" + "\n".join(mismatches))
    return cfg


class ZeroEngine:
    """Owns DDP buffers, the fused AdamW optimizer, LR schedule and loss scaling for one model."""

    def __init__(self, model: torch.nn.Module, ds_config: Dict, dp_group=None, log=print):
        self.cfg = ds_config
        self.module = model
        z = ds_config.get("zero_optimization", {})
        self.stage = int(z.get("stage", 0))
        self.bf16 = bool(ds_config.get("bf16", {}).get("enabled", False))
        self.fp16 = bool(ds_config.get("fp16", {}).get("enabled", False))
        self.ga = int(ds_config.get("gradient_accumulation_steps", 1))
        self.micro_steps = 0
        self.global_steps = 0
        self.skipped_steps = 0
        self.clip = float(ds_config.get("gradient_clipping", 0.0) or 0.0)
        dtype = torch.bfloat16 if self.bf16 else torch.float16 if self.fp16 else torch.float32
        from ..parallel import zero_init as _zi
        with torch.no_grad():  # parameters only: RoPE tables and other buffers stay fp32
            for p in model.parameters():
                if _zi.is_partitioned(p):
                    if p._zi_shard.dtype != dtype:
                        _zi.cast_(p, dtype)
                elif p.dtype != dtype:
                    p.data = p.data.to(dtype)
        if hasattr(model, "cfg"):
            model.cfg.params_dtype = dtype
        bucket = int(z.get("reduce_bucket_size", 5e8)) if not _is_auto(z.get("reduce_bucket_size")) else int(5e8)
        bucket = max(bucket, MIN_BUCKET)
        if self.stage >= 3:
            # Stage 3 gathers / releases parameters per BUCKET, so buckets are at least one
            # transformer block: the HF "auto" reduce_bucket_size (h^2, 0.59 M elements for OPT-125m)
            # would cut a 7 M-parameter layer into 12 gathers, each with its hook bookkeeping.
            blocks = [sum(_zi.logical_numel(p) for p in c.parameters()) for m in model.modules()
                      if isinstance(m, torch.nn.ModuleList) for c in m.children()]
            if blocks:
                bucket = max(bucket, max(blocks))
        off_p = z.get("offload_param", {}) or {}
        self.offload_param = off_p.get("device") in ("cpu", "nvme")
        if self.offload_param and self.stage < 3:
            raise ValueError("offload_param needs zero_optimization.stage 3")
        if off_p.get("device") == "nvme":
            log("[zero] offload_param nvme: shards kept in pinned host memory instead")
        off_o = z.get("offload_optimizer", {}) or {}
        self.offload_optimizer = off_o.get("device") in ("cpu", "nvme")
        self.ddp = DistributedDataParallel(model, dp_group=dp_group, grad_dtype=torch.float32, bucket_size=bucket,
                                           overlap_grad_reduce=bool(z.get("overlap_comm", True)),
                                           use_distributed_optimizer=self.stage >= 1,
                                           overlap_param_gather=self.stage in (1, 2),
                                           zero_stage=max(self.stage, 1))
        self.partitioner = None
        if self.stage >= 3:
            from ..parallel.zero3 import ZeroParamPartitioner

            def _num(key, default):
                v = z.get(key, default)
                return default if _is_auto(v) else int(v)
            self.partitioner = ZeroParamPartitioner(
                self.ddp, persistence_threshold=_num("stage3_param_persistence_threshold", 100_000),
                prefetch_numel=_num("stage3_prefetch_bucket_size", 50_000_000), offload=self.offload_param,
                max_live_numel=_num("stage3_max_live_parameters", 1_000_000_000))
            mem = self.partitioner.param_memory_numel()
            log(f"[zero] stage 3: {self.ddp.numel / 1e9:.2f} B params "
                f"({'partitioned at construction' if self.ddp._zero_init else 'resident before partitioning'}) -> shard {mem['shard'] / 1e9:.3f} B elements on {mem['device']} "
                f"+ {mem['persistent'] / 1e6:.2f} M persistent; grad shard {self.ddp.grad_memory_numel() / 1e9:.3f} B")
        ocfg = ds_config.get("optimizer", {"type": "AdamW", "params": {}})
        otype = ocfg.get("type", "AdamW").lower()
        if otype not in ("adamw", "adam", "fusedadam", "cpuadam"):
            raise ValueError(f"optimizer type {ocfg.get('type')} not supported (AdamW/Adam)")
        op = ocfg.get("params", {})
        adamw = otype == "adamw" or bool(op.get("adam_w_mode", True))
        scaler = None
        dev = next(model.parameters()).device
        if self.fp16:
            f = ds_config["fp16"]
            ls = f.get("loss_scale", 0)
            if ls:
                scaler = ConstantLossScaler(float(ls), device=dev)
            else:
                scaler = DynamicLossScaler(initial_scale=2.0 ** f.get("initial_scale_power", 16),
                                           growth_interval=f.get("loss_scale_window", 1000),
                                           hysteresis=f.get("hysteresis", 2),
                                           min_scale=f.get("min_loss_scale", 1), device=dev)
        opt_cls = MixedPrecisionAdam
        if self.offload_optimizer:
            from ..optim.cpu_adam import CPUOffloadAdam
            opt_cls = CPUOffloadAdam
        self.optimizer = opt_cls(self.ddp, lr=float(op.get("lr", 1e-3)), betas=tuple(op.get("betas", (0.9, 0.999))),
                                 eps=float(op.get("eps", 1e-8)), weight_decay=float(op.get("weight_decay", 0.0)),
                                 adamw=adamw, clip_grad=self.clip, loss_scaler=scaler)
        self.lr_scheduler = None
        scfg = ds_config.get("scheduler")
        if scfg:
            sp = scfg.get("params", {})
            t = scfg.get("type")
            if t == "WarmupDecayLR":
                self.lr_scheduler = WarmupDecayLR(self.optimizer, sp["total_num_steps"], sp.get("warmup_min_lr", 0.0),
                                                  sp.get("warmup_max_lr", 1e-3), sp.get("warmup_num_steps", 1000),
                                                  sp.get("warmup_type", "log"))
            elif t == "WarmupLR":
                self.lr_scheduler = WarmupDecayLR(self.optimizer, 1 << 62, sp.get("warmup_min_lr", 0.0),
                                                  sp.get("warmup_max_lr", 1e-3), sp.get("warmup_num_steps", 1000),
                                                  sp.get("warmup_type", "log"))
            elif t == "WarmupCosineLR":
                self.lr_scheduler = LambdaWarmupScheduler(self.optimizer, "cosine", float(op.get("lr", 1e-3)),
                                                          sp.get("warmup_num_steps", 0), sp["total_num_steps"])
            else:
                raise ValueError(f"scheduler {t} not supported")
        self.steps_per_print = int(ds_config.get("steps_per_print", 10))

    # ------------------------------------------------------------------ training API
    def set_scheduler(self, sched):
        self.lr_scheduler = sched

    def is_gradient_accumulation_boundary(self):
        return (self.micro_steps + 1) % self.ga == 0

    def no_sync(self):
        return self.ddp.no_sync()

    def forward(self, *a, **k):
        return self.module(*a, **k)

    __call__ = forward

    def backward(self, loss, window: bool = False):
        """Scale by 1/GA (and the fp16 loss scale); reduction is launched from the grad hooks on
        the last micro-batch of an accumulation window. ``window``: ``loss`` already covers a
        whole accumulation window (the GA micro-batches fused into one batch, each weighted 1/GA):
        no 1/GA scaling, and this backward is the window's synchronising pass."""
        if window:
            from ..parallel.tensor_parallel import DEFERRED_WGRAD
            DEFERRED_WGRAD.hold = False
            self.micro_steps = (self.micro_steps // self.ga) * self.ga + self.ga - 1
            if self.optimizer.scaler is not None:
                loss = loss * self.optimizer.scaler.scale
            loss.backward()
            return
        loss = loss / self.ga
        if self.optimizer.scaler is not None:
            loss = loss * self.optimizer.scaler.scale
        boundary = self.is_gradient_accumulation_boundary()
        if self._hold_wgrad():
            # the window's weight-gradient GEMMs meet in the deferred queue and run once over all
            # of its tokens in the boundary pass (parallel/tensor_parallel.DeferredWgrad.hold)
            from ..parallel.tensor_parallel import DEFERRED_WGRAD
            DEFERRED_WGRAD.hold = not boundary
        ctx = nullcontext() if boundary else self.ddp.no_sync()
        with ctx:
            loss.backward()

    def _hold_wgrad(self) -> bool:
        """Merged accumulation-window wgrad (parallel/tensor_parallel.accumulation_window_ok)."""
        if self.ga <= 1 or self.partitioner is not None:
            return False
        from ..parallel.tensor_parallel import accumulation_window_ok
        return accumulation_window_ok([self.ddp])

    def step(self):
        """Optimizer step at the accumulation boundary; returns the grad-norm tensor or None."""
        boundary = self.is_gradient_accumulation_boundary()
        self.micro_steps += 1
        if not boundary:
            return None
        self.ddp.finish_grad_sync()
        gn = self.optimizer.step()
        # DeepSpeed skips the LR schedule on an fp16 overflow step (_take_model_step); the check
        # costs one host sync per boundary step and only runs with a loss scaler.
        overflow = self.optimizer.scaler is not None and bool(self.optimizer.found_inf.item())
        if overflow:
            self.skipped_steps += 1
        elif self.lr_scheduler is not None:
            self.lr_scheduler.step()
        self.ddp.zero_grad_buffer()
        self.global_steps += 1
        return gn

    def gathered_params(self):
        """Context with every parameter materialised (ZeRO-3 saves / evaluation); no-op below 3."""
        return self.ddp.gathered_params()

    def get_lr(self):
        return [self.optimizer.lr]

    def wait_for_params(self):
        """Finish the in-flight (overlapped) ZeRO param all-gather before reading parameters
        outside a forward pass (saving, evaluation on another module, returning weights)."""
        self.ddp.wait_param_gather()

    # ------------------------------------------------------------------ checkpoints
    def _param_meta(self):
        names = {id(p): n for n, p in self.module.named_parameters()}
        meta = {}
        for p in self.ddp.params:
            o, n = self.ddp.param_index[id(p)]
            meta[names[id(p)]] = (o, n, tuple(self.ddp.shapes[id(p)][0]))
        return meta

    def save_checkpoint(self, save_dir: str, tag: Optional[str] = None, client_state: Optional[Dict] = None):
        self.wait_for_params()
        tag = tag or f"global_step{self.global_steps}"
        d = os.path.join(save_dir, tag)
        rank = dist.get_rank() if dist.is_initialized() else 0
        os.makedirs(d, exist_ok=True)
        dp_rank = self.ddp.dp_rank
        pre = "bf16_" if self.bf16 else ""
        opt = {"optimizer_state_dict": self.optimizer.state_dict(), "zero_stage": self.stage,
               "partition_count": self.ddp.dp, "ds_config": self.cfg, "ds_version": "smdt-zero-1"}
        _atomic_save(opt, os.path.join(d, f"{pre}zero_pp_rank_{dp_rank}_mp_rank_00_optim_states.pt"))
        with self.gathered_params():
            module_sd = {k: v.detach().cpu().clone() for k, v in self.module.state_dict().items()} if rank == 0 else None
        if rank == 0:
            state = {"module": module_sd,
                     "param_meta": self._param_meta(), "numel": self.ddp.numel,
                     "buffer_names": [], "global_steps": self.global_steps, "micro_steps": self.micro_steps,
                     "lr_scheduler": self.lr_scheduler.state_dict() if self.lr_scheduler else None,
                     "dp_world_size": self.ddp.dp, "mp_world_size": 1, "ds_config": self.cfg,
                     "client_state": client_state or {}}
            _atomic_save(state, os.path.join(d, "mp_rank_00_model_states.pt"))
        if dist.is_initialized():
            dist.barrier()
        if rank == 0:
            with open(os.path.join(save_dir, "latest"), "w") as f:
                f.write(tag)
            _write_zero_to_fp32_script(save_dir)

    def load_checkpoint(self, load_dir: str, tag: Optional[str] = None, load_optimizer_states: bool = True):
        if tag is None:
            with open(os.path.join(load_dir, "latest")) as f:
                tag = f.read().strip()
        d = os.path.join(load_dir, tag)
        st = torch.load(os.path.join(d, "mp_rank_00_model_states.pt"), map_location="cpu", weights_only=True)
        with torch.no_grad():
            own = dict(self.module.named_parameters())
            if self.partitioner is not None:     # write straight into this rank's shards
                meta = st["param_meta"]
                for k, v in st["module"].items():
                    if k in meta:
                        o, n, _ = meta[k]
                        flat = v.reshape(-1).to(self.ddp.param_dtype)
                        for b in self.ddp.buckets:
                            s0, e0 = self.ddp.shard_range(b)
                            lo, hi = max(o, s0), min(o + n, e0)
                            if lo < hi:
                                self.ddp.param_data[lo:hi].copy_(flat[lo - o:hi - o])
                self.ddp.all_gather_params()
            else:
                for k, v in st["module"].items():
                    if k in own:
                        own[k].copy_(v)
        self.global_steps = int(st["global_steps"])
        self.micro_steps = int(st["micro_steps"])
        if self.lr_scheduler is not None and st.get("lr_scheduler"):
            self.lr_scheduler.load_state_dict(st["lr_scheduler"])
        if load_optimizer_states:
            pre = "bf16_" if self.bf16 else ""
            path = os.path.join(d, f"{pre}zero_pp_rank_{self.ddp.dp_rank}_mp_rank_00_optim_states.pt")
            o = torch.load(path, map_location="cpu", weights_only=True)
            if int(o["partition_count"]) != self.ddp.dp:
                raise ValueError(f"checkpoint has {o['partition_count']} partitions, running with {self.ddp.dp}; "
                                 "consolidate with zero_to_fp32 and load weights only")
            self.optimizer.load_state_dict(o["optimizer_state_dict"])
        else:
            self.optimizer.reload_model_params()
        return d, st.get("client_state", {})


def _atomic_save(obj, path):
    tmp = path + ".tmp"
    torch.save(obj, tmp)
    os.replace(tmp, path)


# ---------------------------------------------------------------------------- zero_to_fp32
def get_fp32_state_dict_from_zero_checkpoint(checkpoint_dir: str, tag: Optional[str] = None) -> Dict[str, torch.Tensor]:
    """Rebuild full fp32 weights from the per-rank optimizer shards (DeepSpeed ``zero_to_fp32``)."""
    if tag is None:
        with open(os.path.join(checkpoint_dir, "latest")) as f:
            tag = f.read().strip()
    d = os.path.join(checkpoint_dir, tag)
    st = torch.load(os.path.join(d, "mp_rank_00_model_states.pt"), map_location="cpu", weights_only=True)
    flat = torch.zeros(int(st["numel"]), dtype=torch.float32)
    filled = torch.zeros(int(st["numel"]), dtype=torch.bool)
    files = sorted(f for f in os.listdir(d) if "zero_pp_rank_" in f and f.endswith("_optim_states.pt"))
    if not files:
        raise FileNotFoundError(f"no ZeRO optimizer shards in {d}")
    for f in files:
        o = torch.load(os.path.join(d, f), map_location="cpu", weights_only=True)["optimizer_state_dict"]
        off = 0
        for s, e in o["pieces"]:
            n = e - s
            flat[s:e] = o["master"][off:off + n].float()
            filled[s:e] = True
            off += n
    out = {}
    for name, (o, n, shape) in st["param_meta"].items():
        if not bool(filled[o:o + n].all()):
            raise ValueError(f"{name}: not covered by the optimizer shards (missing rank files?)")
        out[name] = flat[o:o + n].view(shape).clone()
    for k, v in st["module"].items():  # non-trainable entries / buffers
        out.setdefault(k, v.float() if v.is_floating_point() else v)
    return out


def convert_zero_checkpoint_to_fp32_state_dict(checkpoint_dir: str, output_file: str, tag: Optional[str] = None):
    sd = get_fp32_state_dict_from_zero_checkpoint(checkpoint_dir, tag)
    if output_file.endswith(".safetensors"):
        from safetensors.torch import save_file
        save_file({k: v.contiguous() for k, v in sd.items()}, output_file)
    else:
        torch.save(sd, output_file)
    return output_file


_SCRIPT = '''#!/usr/bin/env python
# Consolidate the ZeRO shards in this directory into one fp32 state dict:
#   python zero_to_fp32.py . pytorch_model.bin      (or model.safetensors)
import sys
from smdt_amd.train.zero import convert_zero_checkpoint_to_fp32_state_dict
if __name__ == "__main__":
    convert_zero_checkpoint_to_fp32_state_dict(sys.argv[1], sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else None)
'''


def _write_zero_to_fp32_script(save_dir):
    p = os.path.join(save_dir, "zero_to_fp32.py")
    if not os.path.exists(p):
        with open(p, "w") as f:
            f.write(_SCRIPT)
        os.chmod(p, 0o755)


def initialize(model, config, dp_group=None, log=print):
    """``deepspeed.initialize``-shaped entry: returns (engine, optimizer, None, lr_scheduler)."""
    eng = ZeroEngine(model, load_ds_config(config), dp_group=dp_group, log=log)
    return eng, eng.optimizer, None, eng.lr_scheduler


if __name__ == "__main__":  # python -m smdt_amd.train.zero <ckpt_dir> <out_file> [tag]
    import sys
    convert_zero_checkpoint_to_fp32_state_dict(sys.argv[1], sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else None)
