"""Megatron-compatible ``pretrain()`` driver.

Flow (same as the reference recipe's ``pretrain(...)`` call, /root/reference/3_training_megatron-lm/
pretrain_gpt.py:143-149):

    initialize_megatron -> args/validate, torch.distributed (RCCL), TP/PP/DP groups, seeds,
                           tokenizer + padded vocab, timers
    setup_model_and_optimizer -> model_provider(pre, post) -> DDP (contiguous bf16/fp32 buffers,
                           bucketed overlapped grad reduction) -> MixedPrecisionAdam (+ZeRO) ->
                           OptimizerParamScheduler; --load
    build data iterators   -> train_valid_test_datasets_provider(num_samples) -> Megatron samplers
    train loop             -> forward/backward schedule (no-pipelining or 1F1B), optimizer step,
                           LR step, training_log every --log-interval (line format of NB3:4347),
                           evaluate every --eval-interval, save every --save-interval, exit hooks
                           (--exit-interval, --exit-duration-in-mins, --exit-signal-handler)

The iteration log is printed by the LAST rank (as in the reference log) and optionally mirrored
to a JSONL metrics sink (--metrics-jsonl) with tokens/s and model TFLOP/s.
"""
from __future__ import annotations

import json
import math
import os
import signal
import sys
import time
from datetime import datetime
from typing import Callable, Optional

import torch
import torch.distributed as dist

from ..comm import init_distributed, print_rank_0, print_rank_last
from ..comm import relay as _relay
from ..data.gpt_dataset import SyntheticGPTDataset, build_pretraining_data_loader
from ..data.tokenizer import build_tokenizer, vocab_size_with_padding
from ..models.gpt import allreduce_word_embedding_grads, gpt_flops_per_token
from ..optim.lr_scheduler import OptimizerParamScheduler
from ..optim.optimizer import ConstantLossScaler, DynamicLossScaler, MixedPrecisionAdam, MixedPrecisionSGD
from ..parallel import state as ps
from ..parallel import tensor_parallel as tp
from ..parallel.distributed import DistributedDataParallel
from ..parallel.random import model_parallel_seed
from . import arguments as A
from .checkpointing import finalize_async_save, load_checkpoint, save_checkpoint
from .schedules import get_forward_backward_func
from .timers import Timers
from .utils import report_memory, unwrap_model
from ..utils.debug import StepWatchdog, collective_check_from_env, maybe_inject_fault


class ModelType:
    encoder_or_decoder = 1
    encoder_and_decoder = 2


_START_TIME = time.time()
_SIGNAL = {"received": False}


def _signal_handler(signum, frame):
    _SIGNAL["received"] = True


def initialize_megatron(extra_args_provider=None, args_defaults=None, ignore_unknown_args=False, argv=None):
    args = A.parse_args(extra_args_provider, ignore_unknown_args, argv)
    rank, local, world, backend = init_distributed(args.distributed_backend, args.distributed_timeout_minutes)
    args.rank, args.world_size, args.local_rank = rank, world, local
    if args.use_checkpoint_args or (args_defaults or {}).get("use_checkpoint_args", False):
        from .checkpointing import load_args_from_checkpoint
        load_args_from_checkpoint(args)
    A.validate_args(args, args_defaults or {})
    ps.initialize_model_parallel(args.tensor_model_parallel_size, args.pipeline_model_parallel_size,
                                 args.virtual_pipeline_model_parallel_size, args.context_parallel_size)
    model_parallel_seed(args.seed, args.data_parallel_random_init)
    from .schedules import set_pipeline_schedule
    set_pipeline_schedule(getattr(args, "pp_schedule", "1f1b"))
    if args.pipeline_model_parallel_size > 1:
        print_rank_0(f"> pipeline schedule: "
                     f"{'interleaved' if args.virtual_pipeline_model_parallel_size else args.pp_schedule}")
    args.mb_calculator = A.MicroBatchCalculator(args.global_batch_size, args.micro_batch_size,
                                                args.data_parallel_size, args.rampup_batch_size)
    print_rank_0(args.mb_calculator.describe())
    args.current_global_batch_size = args.mb_calculator.current
    if args.rampup_batch_size and args.train_samples:
        # Megatron's update_train_iters: iterations while ramping + the rest at the full batch
        consumed, iters = 0, 0
        while consumed < args.train_samples:
            consumed += args.mb_calculator.update(consumed)
            iters += 1
        args.mb_calculator.update(0)
        args.train_iters = iters
    tok = None
    if args.tokenizer_type is not None and not (args.mock_data and args.vocab_file is None):
        tok, padded = build_tokenizer(args.tokenizer_type, args.vocab_file, args.merge_file, args.tokenizer_model,
                                      args.vocab_size, args.make_vocab_size_divisible_by,
                                      args.tensor_model_parallel_size, args.rank)
    else:
        from ..data.tokenizer import NullTokenizer
        tok = NullTokenizer(args.vocab_size or 50257)
        padded = vocab_size_with_padding(tok.vocab_size, args.make_vocab_size_divisible_by,
                                         args.tensor_model_parallel_size)
    args.padded_vocab_size = padded
    A.set_global("args", args)
    A.set_global("tokenizer", tok)
    A.set_global("timers", Timers(args.timing_log_level, args.timing_log_option, roctx=args.profile))
    A.print_args(args)
    if args.exit_signal_handler:
        signal.signal(signal.SIGTERM, _signal_handler)
    print_rank_0(f"time to initialize megatron (seconds): {time.time() - _START_TIME:.3f}")
    print_rank_0(f"[after megatron is initialized] datetime: {datetime.now().strftime('%Y-%m-%d %H:%M:%S')}")
    return args


def get_model(model_provider_func, args):
    st = ps.get_state()
    dev = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")
    if st.pp > 1 and st.virtual_pp is not None and st.virtual_pp > 1:
        # interleaved pipeline: vpp model chunks per rank, one flat DDP buffer over all of them
        chunks = []
        for c in range(st.virtual_pp):
            st.virtual_pp_rank = c
            chunks.append(model_provider_func(pre_process=st.is_first_stage(), post_process=st.is_last_stage()))
        st.virtual_pp_rank = 0
        model = torch.nn.ModuleList(chunks)
    else:
        model = model_provider_func(pre_process=st.is_first_stage(), post_process=st.is_last_stage())
    model = model.to(device=dev, dtype=args.params_dtype)
    n = sum(p.numel() for p in model.parameters())
    if st.dp_rank == 0:
        print(f" > number of parameters on (tensor, pipeline) model parallel rank ({st.tp_rank}, {st.pp_rank}): {n}",
              flush=True)
    grad_dtype = torch.float32 if (args.accumulate_allreduce_grads_in_fp32 or args.params_dtype != torch.float32) \
        else args.params_dtype
    ddp = DistributedDataParallel(model, grad_dtype=grad_dtype, bucket_size=args.ddp_bucket_size,
                                  use_distributed_optimizer=args.use_distributed_optimizer and st.dp * st.cp > 1,
                                  overlap_param_gather=getattr(args, "overlap_param_gather", False))
    return ddp


def setup_model_and_optimizer(model_provider_func, args):
    # --no-gradient-accumulation-fusion: weight gradients are computed, then added to main_grad
    # (instead of the MFMA wgrad kernels accumulating straight into the fp32 buffer)
    tp._FUSED_WGRAD = bool(getattr(args, "gradient_accumulation_fusion", True)) and tp._FUSED_WGRAD
    ddp = get_model(model_provider_func, args)
    scaler = None
    if args.fp16:
        dev = ddp.param_data.device
        scaler = ConstantLossScaler(args.loss_scale, dev) if args.loss_scale else DynamicLossScaler(
            args.initial_loss_scale, args.min_loss_scale, growth_interval=int(args.loss_scale_window),
            hysteresis=args.hysteresis, device=dev)
    if getattr(args, "optimizer", "adam") == "sgd":
        opt = MixedPrecisionSGD(ddp, lr=args.lr, momentum=args.sgd_momentum,
                                weight_decay=args.weight_decay, clip_grad=args.clip_grad,
                                loss_scaler=scaler)
    else:
        opt = MixedPrecisionAdam(ddp, lr=args.lr, betas=(args.adam_beta1, args.adam_beta2),
                                 eps=args.adam_eps, weight_decay=args.weight_decay, adamw=True,
                                 clip_grad=args.clip_grad, loss_scaler=scaler)
    print_rank_0(f"> optimizer: {type(opt).__name__}")
    if args.train_samples:
        # Sample-based training (Megatron's rule, also under --rampup-batch-size, where
        # initialize_megatron derived train_iters): warmup / decay are counted in SAMPLES and the
        # scheduler advances by each step's global batch, so a ramping batch warms up correctly.
        decay = args.lr_decay_samples or args.train_samples
        warm = args.lr_warmup_samples or 0
        if args.lr_warmup_fraction is not None:
            warm = int(args.lr_warmup_fraction * decay)
        wd_steps = args.train_samples
        args.lr_step_unit = "samples"
    else:
        decay = args.lr_decay_iters or args.train_iters
        warm = args.lr_warmup_iters
        if args.lr_warmup_fraction is not None:
            warm = int(args.lr_warmup_fraction * decay)
        wd_steps = args.train_iters or decay
        args.lr_step_unit = "iterations"
    sched = OptimizerParamScheduler(opt, args.lr, args.min_lr, warm, decay, args.lr_decay_style,
                                    args.start_weight_decay, args.end_weight_decay,
                                    wd_steps, args.weight_decay_incr_style,
                                    args.use_checkpoint_opt_param_scheduler, args.override_opt_param_scheduler)
    args.iteration = 0
    args.consumed_train_samples = 0
    args.consumed_valid_samples = 0
    if args.load:
        A.get_timers()("load-checkpoint", log_level=0).start(barrier=True)
        args.iteration = load_checkpoint(ddp, opt, sched, args)
        A.get_timers()("load-checkpoint").stop(barrier=True)
    return ddp, opt, sched


def _cyclic(loader):
    while True:
        for b in loader:
            yield b


def build_train_valid_test_data_iterators(provider: Callable, args):
    st = ps.get_state()
    train_iters = args.train_iters or (args.train_samples // args.global_batch_size)
    eval_iters = (train_iters // args.eval_interval + 1) * args.eval_iters
    n = [train_iters * args.global_batch_size, eval_iters * args.global_batch_size, args.eval_iters * args.global_batch_size]
    print_rank_0("> building train, validation, and test datasets ...")
    print_rank_0(f" > datasets target sizes (minimum size):\n    train:      {n[0]}\n    validation: {n[1]}\n    test:       {n[2]}")
    need = st.tp_rank == 0  # only TP rank 0 reads data; the batch is broadcast across TP
    if args.mock_data or not (args.data_path or args.train_data_path):
        sets = tuple(SyntheticGPTDataset(k, args.seq_length, A.get_tokenizer().vocab_size, args.seed + i)
                     for i, k in enumerate(n))
    else:
        sets = provider(n)
    iters = []
    for i, ds in enumerate(sets):
        if ds is None or not need:
            iters.append(None)
            continue
        consumed = args.consumed_train_samples if i == 0 else 0
        loader = build_pretraining_data_loader(ds, consumed, args.micro_batch_size, args.num_workers)
        iters.append(_cyclic(loader) if (i > 0 or args.dataloader_type == "cyclic") else iter(loader))
    return tuple(iters)


def _tokens_per_iter(args):
    return args.global_batch_size * args.seq_length


_TB = {"writer": None}


def get_tensorboard_writer():
    """The event-file writer of the LAST rank when ``--tensorboard-dir`` is set (Megatron's
    ``_set_tensorboard_writer``), else None."""
    return _TB["writer"]


def _set_tensorboard_writer(args):
    last = (not dist.is_initialized()) or dist.get_rank() == dist.get_world_size() - 1
    if getattr(args, "tensorboard_dir", None) and last and _TB["writer"] is None:
        from ..utils.tensorboard import SummaryWriter
        print("> setting tensorboard ...", flush=True)
        _TB["writer"] = SummaryWriter(args.tensorboard_dir, max_queue=args.tensorboard_queue_size)


def _tensorboard_log(writer, loss_dict, lr, iteration, loss_scale, grad_norm, args, timers):
    """Megatron's scalar set (learning-rate, batch-size, each loss, loss-scale, world-size,
    grad-norm, memory; the ``vs samples`` twins keyed by consumed samples)."""
    samples = args.consumed_train_samples
    if args.log_timers_to_tensorboard:   # collective: every rank calls it
        timers.write(["forward-backward", "optimizer", "batch-generator"], writer, iteration)
    if writer is None:
        return
    if args.log_learning_rate_to_tensorboard:
        writer.add_scalar("learning-rate", lr, iteration)
        writer.add_scalar("learning-rate vs samples", lr, samples)
    if args.log_batch_size_to_tensorboard:
        bs = getattr(args, "current_global_batch_size", args.global_batch_size)
        writer.add_scalar("batch-size", bs, iteration)
        writer.add_scalar("batch-size vs samples", bs, samples)
    for k, v in loss_dict.items():
        writer.add_scalar(k, v, iteration)
        writer.add_scalar(k + " vs samples", v, samples)
    if args.log_loss_scale_to_tensorboard and loss_scale is not None:
        writer.add_scalar("loss-scale", loss_scale, iteration)
        writer.add_scalar("loss-scale vs samples", loss_scale, samples)
    if args.log_world_size_to_tensorboard:
        writer.add_scalar("world-size", dist.get_world_size() if dist.is_initialized() else 1, iteration)
    if grad_norm is not None:
        writer.add_scalar("grad-norm", grad_norm, iteration)
        writer.add_scalar("grad-norm vs samples", grad_norm, samples)
    if args.log_memory_to_tensorboard and torch.cuda.is_available():
        writer.add_scalar("mem-reserved-bytes", torch.cuda.memory_reserved(), iteration)
        writer.add_scalar("mem-allocated-bytes", torch.cuda.memory_allocated(), iteration)
        writer.add_scalar("mem-max-allocated-bytes", torch.cuda.max_memory_allocated(), iteration)


def training_log(loss_dict, total_loss_dict, lr, iteration, loss_scale, report_memory_flag, skipped, grad_norm,
                 args, elapsed_per_iter, model_cfg=None, num_zeros_in_grad=None, params_norm=None):
    timers = A.get_timers()
    if iteration % args.log_interval == 0:
        _relay.check_all()          # no TP-pair exchange timed out (outputs would be NaN)
    if getattr(args, "tensorboard_dir", None) and iteration % args.tensorboard_log_interval == 0:
        _tensorboard_log(get_tensorboard_writer(), loss_dict, lr, iteration, loss_scale, grad_norm, args, timers)
    for k, v in loss_dict.items():
        total_loss_dict[k] = total_loss_dict.get(k, 0.0) + float(v)
    total_loss_dict["skipped"] = total_loss_dict.get("skipped", 0) + int(skipped)
    total_loss_dict["iters"] = total_loss_dict.get("iters", 0) + 1
    if iteration % args.log_interval != 0:
        return report_memory_flag
    n = max(total_loss_dict["iters"] - total_loss_dict["skipped"], 1)
    s = f" iteration {iteration:8d}/{args.train_iters:8d} |"
    s += f" consumed samples: {args.consumed_train_samples:12d} |"
    s += f" elapsed time per iteration (ms): {elapsed_per_iter * 1000.0:.1f} |"
    s += f" learning rate: {lr:.3E} |"
    s += f" global batch size: {getattr(args, 'current_global_batch_size', args.global_batch_size):5d} |"
    for k in sorted(total_loss_dict):
        if k in ("skipped", "iters", "nan"):
            continue
        s += f" {k}: {total_loss_dict[k] / n:.6E} |"
    if loss_scale is not None:
        s += f" loss scale: {loss_scale:.1f} |"
    if grad_norm is not None:
        s += f" grad norm: {grad_norm:.3f} |"
    if num_zeros_in_grad is not None:
        s += f" num zeros: {float(num_zeros_in_grad):.1f} |"
    if params_norm is not None:
        s += f" params norm: {params_norm:.3f} |"
    s += f" number of skipped iterations: {total_loss_dict['skipped']:3d} |"
    s += f" number of nan iterations: {total_loss_dict.get('nan', 0):3d} |"
    tps = _tokens_per_iter(args) / max(elapsed_per_iter, 1e-9)
    if model_cfg is not None:
        s += f" throughput (tokens/s): {tps:.0f} |"
    print_rank_last(s)
    if args.metrics_jsonl and ((not dist.is_initialized()) or dist.get_rank() == dist.get_world_size() - 1):
        rec = {"iteration": iteration, "lr": lr, "elapsed_ms": elapsed_per_iter * 1000.0, "tokens_per_s": tps,
               "grad_norm": grad_norm, "loss_scale": loss_scale, "skipped": total_loss_dict["skipped"]}
        rec.update({k: total_loss_dict[k] / n for k in total_loss_dict if k not in ("skipped", "iters", "nan")})
        if model_cfg is not None:
            ws = dist.get_world_size() if dist.is_initialized() else 1
            rec["model_tflops_per_gpu"] = tps * gpt_flops_per_token(model_cfg, args.seq_length) / ws / 1e12
        with open(args.metrics_jsonl, "a") as f:
            f.write(json.dumps(rec) + "\n")
    if report_memory_flag:
        st = ps.get_state()
        if st.dp_rank == 0 and st.pp_rank == 0:
            print(report_memory(f"after {iteration} iterations"), flush=True)
        report_memory_flag = False
    timers.log(["forward-backward", "optimizer", "batch-generator"], normalizer=args.log_interval)
    total_loss_dict.clear()
    return report_memory_flag


def empty_unused_memory(args, level: int):
    """Megatron's ``--empty-unused-memory-level``: 1 returns the caching allocator's free blocks to
    the device after each forward-backward (and each eval iteration), 2 also after the optimizer
    step. Costs allocator re-warm-up; for runs that share the GPU or sit at the HBM limit."""
    if int(getattr(args, "empty_unused_memory_level", 0) or 0) >= level and torch.cuda.is_available():
        torch.cuda.empty_cache()


def train_step(forward_step_func, data_iterator, model, optimizer, scheduler, args):
    timers = A.get_timers()
    model.zero_grad_buffer()
    fb = get_forward_backward_func()
    st = ps.get_state()
    seq = args.seq_length // getattr(args, "context_parallel_size", 1)
    seq = seq // args.tensor_model_parallel_size if args.sequence_parallel else seq
    timers("forward-backward", log_level=1).start(barrier=args.barrier_with_L1_time)
    scaler = getattr(optimizer, "scaler", None)
    losses = fb(forward_step_func, data_iterator, model, args.num_micro_batches,
                tensor_shape=(seq, args.micro_batch_size, args.hidden_size), dtype=args.params_dtype,
                grad_scale=scaler.scale if scaler is not None else None)
    model.finish_grad_sync()
    allreduce_word_embedding_grads(unwrap_model(model))
    empty_unused_memory(args, 1)
    timers("forward-backward").stop()
    timers("optimizer", log_level=1).start(barrier=args.barrier_with_L1_time)
    samples = getattr(args, "lr_step_unit", "iterations") == "samples"
    lr = scheduler.step(getattr(args, "current_global_batch_size", args.global_batch_size) if samples else 1)
    # --log-num-zeros-in-grad: counted on the reduced gradients before the update (an overlapped
    # optimizer re-zeroes them as it goes), on the iterations that log
    if getattr(args, "log_num_zeros_in_grad", False) and hasattr(optimizer, "num_zeros_in_grad") \
            and (getattr(args, "iteration", 0) + 1) % args.log_interval == 0:
        optimizer.last_num_zeros = optimizer.num_zeros_in_grad()
    grad_norm = optimizer.step(lr)
    empty_unused_memory(args, 2)
    timers("optimizer").stop()
    out = {}
    if st.is_last_stage(ignore_virtual=True) and losses:
        for k in losses[0]:
            out[k] = torch.stack([l[k].float().view(-1)[0] for l in losses]).mean()
    return out, lr, grad_norm


def evaluate(forward_step_func, data_iterator, model, args, verbose=False):
    model.eval()
    totals = {}
    fb = get_forward_backward_func()
    seq = args.seq_length // getattr(args, "context_parallel_size", 1)
    seq = seq // args.tensor_model_parallel_size if args.sequence_parallel else seq
    with torch.no_grad():
        for _ in range(args.eval_iters):
            losses = fb(forward_step_func, data_iterator, model, args.num_micro_batches, forward_only=True,
                        tensor_shape=(seq, args.micro_batch_size, args.hidden_size), dtype=args.params_dtype)
            for l in losses:
                for k, v in l.items():
                    totals[k] = totals.get(k, 0.0) + float(v)
            args.consumed_valid_samples += args.global_batch_size
            empty_unused_memory(args, 1)
    model.train()
    n = max(args.eval_iters * args.num_micro_batches, 1)
    return {k: v / n for k, v in totals.items()}


def evaluate_and_print_results(prefix, forward_step_func, data_iterator, model, args):
    res = evaluate(forward_step_func, data_iterator, model, args)
    s = f" validation loss at {prefix} | "
    writer = get_tensorboard_writer()
    for k, v in res.items():
        s += f"{k} value: {v:.6E} | {k} PPL: {math.exp(min(20, v)):.6E} | "
        if writer is not None:
            writer.add_scalar(f"{k} validation", v, args.iteration)
            writer.add_scalar(f"{k} validation vs samples", v, args.consumed_train_samples)
            if args.log_validation_ppl_to_tensorboard:
                writer.add_scalar(f"{k} validation ppl", math.exp(min(20, v)), args.iteration)
    if writer is not None:
        writer.flush()
    length = len(s) + 1
    print_rank_last("-" * length)
    print_rank_last(s)
    print_rank_last("-" * length)
    return res


def _profiler(args, iteration, start: bool):
    if not args.profile or not torch.cuda.is_available():
        return
    rank = dist.get_rank() if dist.is_initialized() else 0
    if rank not in args.profile_ranks:
        return
    try:
        import ctypes
        hip = ctypes.CDLL("libamdhip64.so")
        if start and iteration == args.profile_step_start:
            hip.hipProfilerStart()
        if (not start) and iteration == args.profile_step_end:
            hip.hipProfilerStop()
    except OSError:
        pass


def train(forward_step_func, model, optimizer, scheduler, train_iter, valid_iter, args, model_cfg=None):
    timers = A.get_timers()
    model.train()
    iteration = args.iteration
    total = {}
    report_mem = True
    print_rank_0("training ...")
    t_last = time.time()
    it_since = 0
    watchdog_s = float(os.environ.get("SMDT_STEP_TIMEOUT", "0") or 0)
    while iteration < args.train_iters:
        _profiler(args, iteration, True)
        maybe_inject_fault(iteration + 1)
        mbc = getattr(args, "mb_calculator", None)
        if mbc is not None:   # --rampup-batch-size: micro-batches per step follow consumed samples
            args.current_global_batch_size = mbc.update(args.consumed_train_samples)
            args.num_micro_batches = mbc.num_micro_batches
        else:
            args.current_global_batch_size = args.global_batch_size
        with StepWatchdog(watchdog_s):
            loss_dict, lr, grad_norm = train_step(forward_step_func, train_iter, model, optimizer, scheduler, args)
        collective_check_from_env(iteration + 1)
        iteration += 1
        it_since += 1
        args.iteration = iteration
        args.consumed_train_samples += args.current_global_batch_size
        _profiler(args, iteration, False)
        if iteration % args.log_interval == 0:
            if torch.cuda.is_available():
                torch.cuda.synchronize()
            now = time.time()
            elapsed = (now - t_last) / it_since
            t_last, it_since = now, 0
            # bf16 runs have no scaler, but the Adam kernel still skips a step with inf / nan grads
            fi = int(optimizer.found_inf.item()) if hasattr(optimizer, "found_inf") else 0
            ls = float(optimizer.scaler.scale.item()) if optimizer.scaler is not None else None
            gn = float(grad_norm.item()) if grad_norm is not None else None
            if gn is not None and not math.isfinite(gn):
                total["nan"] = total.get("nan", 0) + 1
            # --log-num-zeros-in-grad / --log-params-norm (collective over the grad-norm groups:
            # every rank reaches this log point)
            nz = getattr(optimizer, "last_num_zeros", None) if getattr(args, "log_num_zeros_in_grad", False) else None
            pn = optimizer.params_norm() if (getattr(args, "log_params_norm", False)
                                             and hasattr(optimizer, "params_norm")) else None
            report_mem = training_log({k: float(v) for k, v in loss_dict.items()}, total, lr, iteration, ls,
                                      report_mem, fi, gn, args, elapsed, model_cfg, nz, pn)
            if getattr(args, "async_save", False):
                finalize_async_save(blocking=False)   # tracker once every rank's writer is done
        # (TP ranks > 0 hold no iterator: get_batch broadcasts from TP rank 0, so all ranks evaluate)
        if args.eval_interval and iteration % args.eval_interval == 0 and args.do_valid:
            evaluate_and_print_results(f"iteration {iteration}", forward_step_func, valid_iter, model, args)
        saved = False
        if args.save and args.save_interval and iteration % args.save_interval == 0:
            timers("save-checkpoint", log_level=0).start(barrier=True)
            save_checkpoint(iteration, model, optimizer, scheduler, args)
            timers("save-checkpoint").stop(barrier=True)
            timers.log(["save-checkpoint"])
            saved = True
        if args.exit_signal_handler and _SIGNAL["received"]:
            if args.save and not saved:
                save_checkpoint(iteration, model, optimizer, scheduler, args)
            finalize_async_save(blocking=True)
            print_rank_0("exiting program after receiving SIGTERM.")
            sys.exit(0)
        if args.exit_duration_in_mins:
            done = torch.tensor([int((time.time() - _START_TIME) / 60.0 > args.exit_duration_in_mins)])
            if dist.is_initialized():
                if torch.cuda.is_available() and dist.get_backend() in ("nccl", "smddp"):
                    done = done.cuda()
                dist.all_reduce(done, op=dist.ReduceOp.MAX)
            if done.item():
                if args.save and not saved:
                    save_checkpoint(iteration, model, optimizer, scheduler, args)
                finalize_async_save(blocking=True)
                print_rank_0(f"exiting program after {args.exit_duration_in_mins} minutes")
                sys.exit(0)
        if args.exit_interval and iteration % args.exit_interval == 0:
            if args.save and not saved:
                save_checkpoint(iteration, model, optimizer, scheduler, args)
            finalize_async_save(blocking=True)
            print_rank_0(f"exiting program at iteration {iteration}")
            sys.exit(0)
    return iteration


def pretrain(train_valid_test_dataset_provider, model_provider, model_type, forward_step_func,
             process_non_loss_data_func=None, extra_args_provider=None, args_defaults=None, argv=None):
    args = initialize_megatron(extra_args_provider, args_defaults, argv=argv)
    _set_tensorboard_writer(args)
    from .schedules import configure_p2p
    configure_p2p(args)   # --overlap-p2p-communication / --no-scatter-gather-tensors-in-pipeline
    timers = A.get_timers()
    timers("model-and-optimizer-setup", log_level=0).start(barrier=True)
    model, optimizer, scheduler = setup_model_and_optimizer(model_provider, args)
    timers("model-and-optimizer-setup").stop()
    print_rank_0(f"[after model, optimizer, and learning rate scheduler are built] datetime: "
                 f"{datetime.now().strftime('%Y-%m-%d %H:%M:%S')}")
    timers("train/valid/test-data-iterators-setup", log_level=0).start(barrier=True)
    train_iter, valid_iter, test_iter = build_train_valid_test_data_iterators(train_valid_test_dataset_provider, args)
    # Only TP rank 0 reads data: broadcast which splits exist to the rest of the TP group.
    st = ps.get_state()
    flags = torch.tensor([int(valid_iter is not None), int(test_iter is not None)], dtype=torch.long)
    if st.tp > 1 and st.tp_group is not None:
        if torch.cuda.is_available() and dist.get_backend() in ("nccl", "smddp"):
            flags = flags.cuda()
        dist.broadcast(flags, st.tp_ranks[0], group=st.tp_group)
    args.do_valid, args.do_test = bool(flags[0].item()), bool(flags[1].item())
    timers("train/valid/test-data-iterators-setup").stop()
    print_rank_0(f"[after dataloaders are built] datetime: {datetime.now().strftime('%Y-%m-%d %H:%M:%S')}")
    timers.log(["model-and-optimizer-setup", "train/valid/test-data-iterators-setup"], barrier=True)
    core = unwrap_model(model)
    model_cfg = getattr(core[0] if isinstance(core, torch.nn.ModuleList) else core, "cfg", None)
    iteration = 0
    if not args.skip_train and args.train_iters:
        iteration = train(forward_step_func, model, optimizer, scheduler, train_iter, valid_iter, args, model_cfg)
        print_rank_0(f"[after training is done] datetime: {datetime.now().strftime('%Y-%m-%d %H:%M:%S')}")
        if args.save and iteration % (args.save_interval or 10 ** 12) != 0:
            save_checkpoint(iteration, model, optimizer, scheduler, args)
        finalize_async_save(blocking=True)
    if args.do_valid and args.eval_iters > 0:
        evaluate_and_print_results(f"iteration {iteration} on validation set", forward_step_func, valid_iter, model,
                                   args)
    if args.do_test and args.eval_iters > 0:
        evaluate_and_print_results(f"iteration {iteration} on test set", forward_step_func, test_iter, model, args)
    if get_tensorboard_writer() is not None:
        get_tensorboard_writer().flush()
    return model, optimizer
