"""HF-``Trainer``-compatible supervised fine-tuning loop on the MI355X stack.

The Alpaca recipe does ``Trainer(model, tokenizer, args, **data_module).train(); save_state();
save_model(output_dir)`` (/root/reference/4_training_alpaca_deepspeed/train.py:243-246). This
``Trainer`` keeps that surface and HF's observable behaviour:

* epochs / ``max_steps`` accounting (``max_steps = ceil(epochs * (len(loader) // GA))``), seeded
  per-epoch shuffling over ranks, gradient accumulation, clipping, AdamW + LR schedule (HF
  ``lr_scheduler_type`` or the DeepSpeed ``scheduler`` block);
* log lines ``{'loss': …, 'learning_rate': …, 'epoch': …}`` every ``logging_steps`` (loss averaged
  over ranks and steps since the last log) and the final
  ``{'train_runtime', 'train_samples_per_second', 'train_steps_per_second', 'train_loss', 'epoch'}``
  summary computed the way HF does (NB4:2306 is the reference's);
* ``checkpoint-N/`` every ``save_steps`` with ``save_total_limit`` rotation, containing the HF model
  (config.json + model.safetensors), tokenizer, ``trainer_state.json``, ``training_args.json``,
  per-rank RNG state, and the DeepSpeed-layout ZeRO checkpoint (``global_stepN/``, ``latest``,
  ``zero_to_fp32.py``); ``resume_from_checkpoint`` restores all of it.

Everything runs through ``ZeroEngine`` (flat fp32 grads, bucketed RCCL reduce-scatter overlapped
with backward, fused AdamW HIP kernel on the shard, bf16 param all-gather) and the model's HIP
kernels (flash attention, fused norm/residual, fused CE). No host synchronisation per micro-batch.
"""
from __future__ import annotations

import glob
import contextlib
import json
import math
import os
import random
import shutil
import time
from typing import Dict, Optional

import numpy as np
import torch
import torch.distributed as dist

from ..comm import init_distributed
from ..data.sft import DistributedRandomSampler, LengthGroupedSampler
from ..optim.lr_scheduler import LambdaWarmupScheduler
from ..parallel import state as ps
from .zero import ZeroEngine, load_ds_config, resolve_ds_config
from ..utils.debug import collective_check_from_env, maybe_inject_fault

PREFIX_CHECKPOINT_DIR = "checkpoint"
TRAINER_STATE_NAME = "trainer_state.json"


def setup_distributed(args=None, backend: str = "nccl"):
    """Init the process group (one process per GPU) + a TP=PP=1 model-parallel state; returns
    (rank, local_rank, world, device). Call before building the model."""
    if dist.is_initialized():
        rank, world = dist.get_rank(), dist.get_world_size()
        local = int(os.environ.get("LOCAL_RANK", "0"))
        if torch.cuda.is_available():
            # a caller-initialised group may not have selected this rank's device
            torch.cuda.set_device(local % torch.cuda.device_count())
    else:  # single process: no process group is created
        # SMDT_DIST_BACKEND=gloo: one-GPU rehearsal of the multi-rank path (RCCL refuses two ranks
        # on one device)
        rank, local, world, _ = init_distributed(os.environ.get("SMDT_DIST_BACKEND", backend))
    emu = int(os.environ.get("SMDT_EMULATE_DP", "0") or 0)
    if emu > 1 and world == 1:
        # timing: this process does ONE data-parallel rank's work of an emu-GPU ZeRO job — its own
        # micro-batches, its 1/emu optimizer shard, its share of the gradient reduce-scatter /
        # parameter all-gather as local copies (parallel/state.initialize_emulated_tensor_parallel)
        ps.initialize_emulated_tensor_parallel(1, emu)
    elif not ps.model_parallel_is_initialized():
        ps.initialize_model_parallel(1, 1)
    # the device init_distributed selected (local_rank modulo the visible devices)
    dev = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")
    if args is not None:
        args.local_rank = local
    return rank, local, world, dev


MI355X_BF16_PEAK_TFLOPS = 2500.0   # dense bf16 MFMA (MI355X_MICROARCH.md: ~2.5 PF dense)

class TrainerState(dict):
    pass


class Trainer:
    def __init__(self, model, tokenizer=None, args=None, train_dataset=None, eval_dataset=None, data_collator=None,
                 ds_config: Optional[Dict] = None):
        self.model = model
        self.tokenizer = tokenizer
        self.args = args
        self.train_dataset = train_dataset
        self.eval_dataset = eval_dataset
        self.data_collator = data_collator
        self.rank, self.local_rank, self.world, self.device = setup_distributed(args)
        self.is_main = self.rank == 0
        self._ds_raw = load_ds_config(ds_config if ds_config is not None else args.deepspeed)
        self.state = TrainerState(log_history=[], global_step=0, epoch=0.0, max_steps=0, num_train_epochs=0,
                                  total_flos=0.0, train_batch_size=args.per_device_train_batch_size,
                                  is_world_process_zero=self.is_main, logging_steps=args.logging_steps,
                                  save_steps=args.save_steps)
        if args.tf32 is not None and torch.cuda.is_available():
            torch.backends.cuda.matmul.allow_tf32 = bool(args.tf32)
            torch.backends.cudnn.allow_tf32 = bool(args.tf32)
        if args.gradient_checkpointing:
            cfg = model.cfg
            cfg.recompute_granularity, cfg.recompute_method, cfg.recompute_num_layers = "full", "uniform", 1
        self._set_seed(args.seed)
        self.engine: Optional[ZeroEngine] = None

    # ------------------------------------------------------------------ utils
    def log(self, logs: Dict):
        logs = dict(logs)
        if "epoch" in logs or self.state["epoch"] is not None:
            logs.setdefault("epoch", round(self.state["epoch"], 2))
        self.state["log_history"].append({**logs, "step": self.state["global_step"]})
        if self.is_main:
            print(logs, flush=True)
            if self.args.metrics_jsonl:
                with open(self.args.metrics_jsonl, "a") as f:
                    f.write(json.dumps({**logs, "step": self.state["global_step"]}) + "\n")

    def _set_seed(self, seed):
        random.seed(seed)
        np.random.seed(seed)
        torch.manual_seed(seed)

    def _build_loader(self, dataset, batch_size, shuffle=True):
        a = self.args
        if a.group_by_length and hasattr(dataset, "lengths") and shuffle:
            sampler = LengthGroupedSampler(dataset.lengths(), batch_size * 1, self.rank, self.world,
                                           a.data_seed if a.data_seed is not None else a.seed)
        else:
            sampler = DistributedRandomSampler(len(dataset), self.rank, self.world,
                                               a.data_seed if a.data_seed is not None else a.seed, shuffle)
        loader = torch.utils.data.DataLoader(dataset, batch_size=batch_size, sampler=sampler,
                                             collate_fn=self.data_collator, num_workers=a.dataloader_num_workers,
                                             pin_memory=a.dataloader_pin_memory and self.device.type == "cuda",
                                             drop_last=a.dataloader_drop_last)
        return loader, sampler

    def _setup_engine(self, max_steps):
        a = self.args
        hidden = self.model.cfg.hidden_size
        if self._ds_raw:
            cfg = resolve_ds_config(self._ds_raw, a, hidden, self.world, max_steps)
        else:  # plain HF Trainer defaults: AdamW (torch), linear schedule, no ZeRO
            cfg = {"bf16": {"enabled": a.bf16}, "fp16": {"enabled": a.fp16},
                   "optimizer": {"type": "AdamW", "params": {"lr": a.learning_rate,
                                                             "betas": [a.adam_beta1, a.adam_beta2],
                                                             "eps": a.adam_epsilon, "weight_decay": a.weight_decay}},
                   "gradient_accumulation_steps": a.gradient_accumulation_steps,
                   "gradient_clipping": a.max_grad_norm, "zero_optimization": {"stage": 0}}
        self.ds_config = cfg
        self.model.to(self.device)
        self.engine = ZeroEngine(self.model, cfg, log=self._log0)
        if self.engine.lr_scheduler is None:
            self.engine.set_scheduler(LambdaWarmupScheduler(self.engine.optimizer, a.lr_scheduler_type,
                                                            a.learning_rate, a.get_warmup_steps(max_steps),
                                                            max_steps))
        self._log0(f"[zero] stage {self.engine.stage}, dtype "
                   f"{'bf16' if self.engine.bf16 else 'fp16' if self.engine.fp16 else 'fp32'}, "
                   f"world {self.world}, {sum(math.prod(sh) for sh, _ in self.engine.ddp.shapes.values()) / 1e6:.1f} M params, "
                   f"{len(self.engine.ddp.buckets)} grad buckets")

    def _log0(self, msg):
        if self.is_main:
            print(msg, flush=True)

    # fraction of the free device memory a fused accumulation window may take for its activations
    FUSE_MEM_FRACTION = 0.6

    def _fuse_decision(self, window) -> bool:
        """``_window_fits`` agreed across the data-parallel group (MIN of one int per window).
        ZeRO-2 reduce-scatters its buckets on every micro-batch and ZeRO-3 all-gathers parameters
        on every forward, so a rank that ran a window unfused would issue GA times the
        collectives of a rank that fused it: each rank's own token count and free memory must
        not decide alone. One 4-byte all-reduce per accumulation window."""
        ok = self._window_fits(window)
        ddp = getattr(getattr(self, "engine", None), "ddp", None)
        from ..comm import loopback as _lb
        if ddp is not None and ddp.dp > 1 and not _lb.is_loopback(ddp.dp_group):
            # (a loopback group is ONE process emulating a rank, SMDT_EMULATE_DP: its own decision)
            dev = self.device if self.device.type == "cuda" and dist.get_backend(ddp.dp_group) != "gloo" \
                else torch.device("cpu")
            t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MIN, group=ddp.dp_group)
            ok = bool(t.item())
        return ok

    def _window_fits(self, window) -> bool:
        """Whether GA micro-batches fused into one batch fit in free device memory: an upper
        estimate of the activations autograd keeps for the fused batch (bf16 per token and layer:
        ~10 h + 3 ffn values — norms, QKV, attention output, residuals, MLP intermediates — plus
        the logits and their fp32 gradient) against SMDT_SFT_FUSE_MEM_FRACTION (0.6) of what
        torch.cuda.mem_get_info reports free now. Always true off-GPU."""
        if self.device.type != "cuda":
            return True
        cfg = getattr(getattr(self.model, "model", None), "cfg", None)
        if cfg is None:
            return True
        toks = sum(int(b["attention_mask"].sum()) if b.get("attention_mask") is not None else b["input_ids"].numel()
                   for b in window)
        rows = sum(b["input_ids"].shape[0] for b in window)
        toks = max(toks, rows * 64)           # padding-free micro-batches round up to 64 rows
        ffn = getattr(cfg, "ffn_hidden_size", None) or 4 * cfg.hidden_size
        per_tok = cfg.num_layers * (10 * cfg.hidden_size + 3 * ffn) * 2 + cfg.padded_vocab_size * 6
        free, _ = torch.cuda.mem_get_info(self.device)
        frac = float(os.environ.get("SMDT_SFT_FUSE_MEM_FRACTION", self.FUSE_MEM_FRACTION))
        return toks * per_tok <= frac * free

    # ------------------------------------------------------------------ train
    def train(self, resume_from_checkpoint=None):
        a = self.args
        resume_from_checkpoint = resume_from_checkpoint or a.resume_from_checkpoint
        loader, sampler = self._build_loader(self.train_dataset, a.per_device_train_batch_size)
        ga = a.gradient_accumulation_steps
        upe = max(len(loader) // ga, 1)
        if a.max_steps > 0:
            max_steps = a.max_steps
            num_epochs = math.ceil(max_steps / upe)
            num_train_samples = max_steps * a.per_device_train_batch_size * ga * self.world
        else:
            max_steps = math.ceil(a.num_train_epochs * upe)
            num_epochs = math.ceil(a.num_train_epochs)
            num_train_samples = int(len(self.train_dataset) * a.num_train_epochs)
        self._setup_engine(max_steps)
        eng = self.engine
        self.state.update(max_steps=max_steps, num_train_epochs=num_epochs)
        start_epoch, skip_batches = 0, 0
        if resume_from_checkpoint:
            if resume_from_checkpoint is True or str(resume_from_checkpoint).lower() == "true":
                resume_from_checkpoint = get_last_checkpoint(a.output_dir)
            if resume_from_checkpoint:
                self._load_checkpoint(resume_from_checkpoint)
                gs = self.state["global_step"]
                start_epoch = gs // upe
                skip_batches = (gs % upe) * ga
                self._log0(f"[sft] resumed from {resume_from_checkpoint} at step {gs}")
        total_bs = a.per_device_train_batch_size * ga * self.world
        self._log0("***** Running training *****")
        self._log0(f"  Num examples = {len(self.train_dataset):,}")
        self._log0(f"  Num Epochs = {num_epochs:,}")
        self._log0(f"  Instantaneous batch size per device = {a.per_device_train_batch_size:,}")
        self._log0(f"  Total train batch size (w. parallel, distributed & accumulation) = {total_bs:,}")
        self._log0(f"  Gradient Accumulation steps = {ga:,}")
        self._log0(f"  Total optimization steps = {max_steps:,}")
        shapes = self.engine.ddp.shapes if self.engine is not None else {}   # ZeRO-3: logical shapes
        nparam = sum(math.prod(shapes[id(p)][0]) if id(p) in shapes else p.numel()
                     for p in self.model.parameters() if p.requires_grad)
        self._log0(f"  Number of trainable parameters = {nparam:,}")
        self.model.train()
        tr_loss = torch.zeros((), dtype=torch.float32, device=self.device)
        total_loss = torch.zeros((), dtype=torch.float32, device=self.device)
        tokens = torch.zeros((), dtype=torch.float64, device=self.device)
        # every non-pad input token (prompt + response): the work the model does, for MFU
        in_tokens = torch.zeros((), dtype=torch.float64, device=self.device)
        pad_tokens = 0         # tokens computed including the padding of each micro-batch
        steady = None          # (time, input tokens) after the first optimizer step (kernel tuning, caches)
        n_seen = 0
        steps_since_log = 0
        last_log_t = t0 = time.time()
        done = self.state["global_step"] >= max_steps
        # MI355X: the GA micro-batches of an accumulation window run as ONE fused batch: the loss is
        # the mean of the micro-batches' own token-means, so the gradient is the one GA accumulated
        # backwards produce — one forward / backward / wgrad per step instead of GA small ones
        # (host-bound at mbs 4). The fused batch holds GA x the activations the DeepSpeed config
        # was sized for, so each window is checked against the free device memory first
        # (``_window_fits``) and runs micro-batch by micro-batch when it would not fit.
        # SMDT_SFT_FUSE_GA=0 always runs them one by one.
        fuse = ga > 1 and os.environ.get("SMDT_SFT_FUSE_GA", "1") == "1"
        window = []
        fused_windows = unfused_windows = 0

        def run(batch, row_groups):
            nonlocal tr_loss, tokens, in_tokens, pad_tokens, n_seen
            ids = batch["input_ids"].to(self.device, non_blocking=True)
            labels = batch["labels"].to(self.device, non_blocking=True)
            maybe_inject_fault(self.state["global_step"] + 1, self.rank)
            # the CPU attention mask lets the model skip the padding (models/hf.py)
            if row_groups is not None:
                loss, _ = self.model(ids, attention_mask=batch.get("attention_mask"), labels=labels,
                                     row_groups=row_groups)
                eng.backward(loss, window=True)
                tr_loss += loss.detach().float()
            else:
                loss, _ = self.model(ids, attention_mask=batch.get("attention_mask"), labels=labels)
                eng.backward(loss)
                tr_loss += loss.detach().float() / ga
            tokens += (labels != -100).sum()
            am = batch.get("attention_mask")
            in_tokens += am.sum() if am is not None else ids.numel()
            pad_tokens += getattr(self.model, "last_computed_tokens", None) or ids.numel()
            n_seen += ids.shape[0]

        try:
            for epoch in range(start_epoch, num_epochs):
                if done:
                    break
                sampler.set_epoch(epoch)
                for step, batch in enumerate(loader):
                    if skip_batches:
                        skip_batches -= 1
                        continue
                    if fuse and batch.get("attention_mask") is not None:
                        window.append(batch)
                        if len(window) < ga:
                            continue
                        if self._fuse_decision(window):
                            fused, row_groups = _fuse_window(window)
                            if fused_windows == 0:
                                self._log0(f"[sft] fused accumulation window: {ga} micro-batches as one batch of "
                                           f"{fused['input_ids'].shape[0]} rows")
                            fused_windows += 1
                            run(fused, row_groups)
                        else:
                            if unfused_windows == 0:
                                self._log0("[sft] accumulation window would not fit as one batch: running its "
                                           "micro-batches one by one")
                            unfused_windows += 1
                            for b in window[:-1]:
                                run(b, None)
                                eng.step()          # (not a boundary)
                            run(window[-1], None)
                        window = []
                    else:
                        run(batch, None)
                    gn = eng.step()
                    if gn is None:
                        continue
                    if steady is None:
                        if self.device.type == "cuda":
                            torch.cuda.synchronize(self.device)
                        steady = (time.time(), float(in_tokens), self.state["global_step"] + 1)
                    collective_check_from_env(self.state["global_step"] + 1)
                    self.state["global_step"] += 1
                    self.state["epoch"] = epoch + (step + 1) / len(loader)
                    steps_since_log += 1
                    gs = self.state["global_step"]
                    if (a.logging_first_step and gs == 1) or (a.logging_steps > 0 and gs % int(a.logging_steps) == 0):
                        t = tr_loss.clone()
                        if self.world > 1:
                            dist.all_reduce(t)
                            t /= self.world
                        total_loss += tr_loss
                        now = time.time()
                        self.log({"loss": round(float(t) / steps_since_log, 4),
                                  "learning_rate": eng.get_lr()[0],
                                  "grad_norm": round(float(gn), 4),
                                  "step_time_s": round((now - last_log_t) / steps_since_log, 4)})
                        tr_loss.zero_()
                        steps_since_log = 0
                        last_log_t = now
                    if a.save_strategy == "steps" and a.save_steps > 0 and gs % int(a.save_steps) == 0:
                        self._save_checkpoint()
                    if a.evaluation_strategy == "steps" and self.eval_dataset is not None and a.eval_steps \
                            and gs % int(a.eval_steps) == 0:
                        self.evaluate()
                    if gs >= max_steps:
                        done = True
                        break
                if a.save_strategy == "epoch":
                    self._save_checkpoint()
                if a.evaluation_strategy == "epoch" and self.eval_dataset is not None:
                    self.evaluate()
        finally:
            # a run stopped inside an accumulation window must not leave held weight gradients
            # (and their dY / X) queued, or the queue in hold mode, for the next user
            from ..parallel.tensor_parallel import reset_wgrad_window
            reset_wgrad_window()
        total_loss += tr_loss
        if self.world > 1:
            dist.all_reduce(total_loss)
            dist.all_reduce(tokens)
            total_loss /= self.world
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        runtime = time.time() - t0
        gs = max(self.state["global_step"], 1)
        if self.world > 1:
            dist.all_reduce(in_tokens)
        metrics = {"train_runtime": round(runtime, 4),
                   "train_samples_per_second": round(num_train_samples / runtime, 3),
                   "train_steps_per_second": round(max_steps / runtime, 3),
                   "train_tokens_per_second": round(float(tokens) / runtime, 1),
                   "train_loss": float(total_loss) / gs}
        # Steady state (after the first optimizer step): input tokens / s and model FLOP/s per GPU
        # with the 6 N + attention count (12 L h s per token, s = mean sequence), and MFU against
        # the dense bf16 MFMA peak of an MI355X (2.5 PF/s).
        if steady is not None and self.state["global_step"] > steady[2]:
            t_s = time.time() - steady[0]
            tok_local = float(in_tokens) / max(1, self.world) - steady[1]
            tps = tok_local * max(1, self.world) / max(t_s, 1e-9)
            cfg = getattr(getattr(self.model, "model", None), "cfg", None)
            attn = 0.0
            if cfg is not None:
                mean_s = float(in_tokens) / max(1.0, float(n_seen * max(1, self.world)))
                attn = 12.0 * cfg.num_layers * cfg.hidden_size * mean_s
            fpt = 6.0 * nparam + attn
            tfl = tps * fpt / max(1, self.world) / 1e12
            metrics.update({"train_input_tokens_per_second": round(tps, 1),
                            "train_model_tflops_per_gpu": round(tfl, 2),
                            "train_mfu": round(tfl / MI355X_BF16_PEAK_TFLOPS, 4),
                            # share of the computed tokens (padded, or padding-free rounded up to
                            # 64) that are real input tokens
                            "train_nonpad_fraction": round(float(in_tokens) / max(1, pad_tokens * max(1, self.world)), 4)})
        st = ps.get_state()
        if getattr(st, "emulated", False) and st.dp > 1:
            # one emulated rank of an st.dp-GPU data-parallel job (SMDT_EMULATE_DP): the job's rate
            # is st.dp times this rank's, plus whatever of the real collectives would not overlap
            metrics["emulated_dp_ranks"] = st.dp
            metrics["predicted_job_train_samples_per_second"] = round(st.dp * metrics["train_samples_per_second"], 3)
            if "train_input_tokens_per_second" in metrics:
                metrics["predicted_job_input_tokens_per_second"] = round(st.dp * metrics["train_input_tokens_per_second"], 1)
        self.log(metrics)
        self.train_metrics = metrics
        return metrics

    @torch.no_grad()
    def evaluate(self, eval_dataset=None):
        ds = eval_dataset or self.eval_dataset
        if ds is None:
            return {}
        loader, _ = self._build_loader(ds, self.args.per_device_eval_batch_size, shuffle=False)
        if self.engine is not None:
            self.engine.wait_for_params()
        self.model.eval()
        tot = torch.zeros(2, dtype=torch.float64, device=self.device)
        for batch in loader:
            ids = batch["input_ids"].to(self.device)
            labels = batch["labels"].to(self.device)
            loss, _ = self.model(ids, labels=labels)
            tot[0] += loss.double()
            tot[1] += 1
        if self.world > 1:
            dist.all_reduce(tot)
        self.model.train()
        m = {"eval_loss": float(tot[0] / tot[1].clamp(min=1))}
        self.log(m)
        return m

    # ------------------------------------------------------------------ saving
    def save_state(self):
        if self.is_main:
            os.makedirs(self.args.output_dir, exist_ok=True)
            with open(os.path.join(self.args.output_dir, TRAINER_STATE_NAME), "w") as f:
                json.dump(dict(self.state), f, indent=2, sort_keys=True)

    def save_model(self, output_dir: Optional[str] = None):
        """HF-format weights (config.json + model.safetensors) + tokenizer + training args from
        rank 0; under ZeRO-3 every rank takes part in gathering the partitioned parameters."""
        out = output_dir or self.args.output_dir
        ctx = contextlib.nullcontext()
        if self.engine is not None:
            self.engine.wait_for_params()
            ctx = self.engine.gathered_params()
        with ctx:
            sd = {k: v.detach().cpu().clone() for k, v in self.model.model.state_dict().items()} \
                if self.is_main and hasattr(self.model, "model") else None
        if self.is_main:
            os.makedirs(out, exist_ok=True)
            self.model.save_pretrained(out, state_dict=sd) if sd is not None else self.model.save_pretrained(out)
            if self.tokenizer is not None and hasattr(self.tokenizer, "save_pretrained"):
                self.tokenizer.save_pretrained(out)
            with open(os.path.join(out, "training_args.json"), "w") as f:
                f.write(self.args.to_json_string())
        if self.world > 1:
            dist.barrier()

    def _rotate_checkpoints(self):
        lim = self.args.save_total_limit
        if not lim or lim <= 0 or not self.is_main:
            return
        cks = sorted_checkpoints(self.args.output_dir)
        for d in cks[: max(0, len(cks) - lim)]:
            shutil.rmtree(d, ignore_errors=True)

    def _save_checkpoint(self):
        gs = self.state["global_step"]
        d = os.path.join(self.args.output_dir, f"{PREFIX_CHECKPOINT_DIR}-{gs}")
        self.save_model(d)
        self.engine.save_checkpoint(d, tag=f"global_step{gs}")
        rng = {"python": list(random.getstate()[1]), "numpy": torch.from_numpy(np.random.get_state()[1].copy()),
               "cpu": torch.get_rng_state()}
        if self.device.type == "cuda":
            rng["cuda"] = torch.cuda.get_rng_state(self.device)
        os.makedirs(d, exist_ok=True)
        torch.save(rng, os.path.join(d, f"rng_state_{self.rank}.pth"))
        if self.is_main:
            with open(os.path.join(d, TRAINER_STATE_NAME), "w") as f:
                json.dump(dict(self.state), f, indent=2, sort_keys=True)
        if self.world > 1:
            dist.barrier()
        self._rotate_checkpoints()

    def _load_checkpoint(self, d):
        self.engine.load_checkpoint(d)
        with open(os.path.join(d, TRAINER_STATE_NAME)) as f:
            self.state.update(json.load(f))
        p = os.path.join(d, f"rng_state_{self.rank}.pth")
        if os.path.exists(p):
            rng = torch.load(p, map_location="cpu", weights_only=True)
            torch.set_rng_state(rng["cpu"])
            if "cuda" in rng and self.device.type == "cuda":
                torch.cuda.set_rng_state(rng["cuda"], self.device)


def sorted_checkpoints(output_dir):
    cks = [d for d in glob.glob(os.path.join(output_dir, f"{PREFIX_CHECKPOINT_DIR}-*")) if os.path.isdir(d)]
    return sorted(cks, key=lambda x: int(x.rsplit("-", 1)[-1]))


def get_last_checkpoint(output_dir):
    cks = sorted_checkpoints(output_dir)
    return cks[-1] if cks else None


def _fuse_window(batches):
    """GA collated micro-batches -> one right-padded batch (pads: id 0, label -100, mask 0) and
    the micro-batch index of every row."""
    L = max(b["input_ids"].shape[1] for b in batches)
    ids, labs, masks, groups = [], [], [], []
    for g, b in enumerate(batches):
        n, l = b["input_ids"].shape
        pad = L - l
        ids.append(torch.nn.functional.pad(b["input_ids"], (0, pad), value=0))
        labs.append(torch.nn.functional.pad(b["labels"], (0, pad), value=-100))
        masks.append(torch.nn.functional.pad(b["attention_mask"].to(torch.bool), (0, pad), value=False))
        groups.append(torch.full((n,), g, dtype=torch.long))
    return (dict(input_ids=torch.cat(ids), labels=torch.cat(labs), attention_mask=torch.cat(masks)),
            torch.cat(groups))
