#!/usr/bin/env python3
"""Headline benchmark: GPT-2 345M Megatron-style pretraining throughput (tokens/s, whole job).

Metric / config from BASELINE.json: "tokens/sec (whole node) GPT-2 345M pretrain at 1/2/4/8
MI355X". Model: 24 layers, hidden 1024, 16 heads, seq 1024, vocab 50257 padded to 50304
(Megatron `--make-vocab-size-divisible-by 128`), random init, synthetic CodeParrot-shaped
tokens. Every timed step is a full training step: forward, backward, bucketed RCCL gradient
reduction (DP), grad clipping and the fused Adam update.

Baseline: the reference publishes no 345M number; its GPT-2-small run reaches ~41 model-TFLOP/s
per A100 (derived from NB3:4718). ``vs_baseline`` compares our model-FLOPs/s per GPU
against that 41 TFLOP/s/GPU, i.e. value / (41e12 * n_gpus / flops_per_token(345M)).

Launch: ``python bench.py`` (1 GPU) or
``python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N``.

Layouts (``--layout``):
  * ``baseline`` (default) — N=8 is BASELINE.json config #3, GPT-2 345M at TP=2 PP=2 DP=2 + SP
    (/root/reference/3_training_megatron-lm/megatron/arguments.py:1002-1005 sets TP/PP; the
    reference's own run, NB3:399-428, used TP4 DP4). N=2 and N=4 run DP-N + ZeRO-1: a TP pair
    shares ONE xGMI link, and at N=2 the sequence-parallel exchanges of a tp2 step (~24.6 GB per
    direction) would take longer than the step's compute, while DP-N moves ~2 GB per step per
    rank across all of a GPU's links and overlaps it with backward (BENCHMARKS.md "link budget").
  * ``dp`` — DP-N + ZeRO-1 at every N (every GPU holds the whole model).
  * ``tp`` — model parallelism first: N=2 tp2, N=4 tp2pp2, N=8 tp2pp2dp2 (+SP).
  ``--tp/--pp`` override any layout. The JSON line names the layout and its parallelism.

Self-explanation (``--comm-stats 1``, default): the JSON line carries ``phase_ms`` — the step split
from CUDA events on the compute stream into forward/backward compute, TP-exchange wait, pipeline
p2p wait + bubble, ZeRO parameter-gather wait, DP gradient sync, optimizer and the device idle gap
between steps (comm/stats.py; the pieces sum to the step) — and ``comm``: per axis (tp / pp / dp /
embd / mp) and op the calls, MB, ms and bus GB/s per step, keyed by the transport that carried them
(rccl / xgmi / relay). They are recorded on two extra steps after the timed ones; nothing is
added to the timed loop.

Scaling is WEAK: every GPU processes ``--seqs-per-gpu`` (64) sequences of 1024 tokens per step
at every N, so global batch = 64 N. A DP replica (tp x pp GPUs) therefore runs 64 tp pp sequences
per step: with pp == 1 as micro-batches of up to 64 sequences (gradient accumulation beyond),
with pp > 1 as micro-batches of up to 32 — 8 micro-batches at tp2pp2: the 1F1B bubble (pp - 1) / m
is 12.5 %, but the larger GEMMs more than pay for it (213 vs 220 ms per rank measured for 16 x 16).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from smdt_amd.comm import init_distributed, relay  # noqa: E402
from smdt_amd.comm import streams as comm_streams  # noqa: E402
from smdt_amd.comm.loopback import link_standin  # noqa: E402
from smdt_amd.models.gpt import GPTModel, allreduce_word_embedding_grads, gpt_flops_per_token, pad_vocab_size  # noqa: E402
from smdt_amd.models.transformer import TransformerConfig  # noqa: E402
from smdt_amd.optim.optimizer import MixedPrecisionAdam  # noqa: E402
from smdt_amd.optim.lr_scheduler import OptimizerParamScheduler  # noqa: E402
from smdt_amd.parallel import state as ps  # noqa: E402
from smdt_amd.parallel.distributed import DistributedDataParallel  # noqa: E402
from smdt_amd.parallel.random import model_parallel_seed  # noqa: E402
from smdt_amd.train.schedules import configure_p2p, get_forward_backward_func, set_pipeline_schedule  # noqa: E402

REF_TFLOPS_PER_GPU = 41.0e12  # reference GPT-2-small on A100 (derived)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--layout", choices=["baseline", "dp", "tp"], default="baseline")
    p.add_argument("--tp", type=int, default=None)
    p.add_argument("--pp", type=int, default=None)
    p.add_argument("--sequence-parallel", type=int, default=None, help="default: on when tp > 1")
    # 64 x 1024 tokens per GPU per step: the 288 GB of HBM holds it without recompute; on one
    # MI355X it measured +3.2 % tokens/s over 32 (profiles/r2_mbs/; 32 was +5 % over 16), it halves
    # the gradient / optimizer bytes per token, and at pp = 2 it gives 8 micro-batches of 32 per step.
    p.add_argument("--seqs-per-gpu", type=int, default=64, help="sequences per GPU per step (weak scaling)")
    p.add_argument("--micro-batch-size", type=int, default=None)
    p.add_argument("--grad-accum", type=int, default=None, help="micro-batches per step per DP rank")
    p.add_argument("--seq-length", type=int, default=1024)
    p.add_argument("--num-layers", type=int, default=24)
    p.add_argument("--hidden-size", type=int, default=1024)
    p.add_argument("--num-attention-heads", type=int, default=16)
    p.add_argument("--vocab-size", type=int, default=50257)
    # per-rank shape emulation on one GPU (benchmarks/predict_scaling.py): a TP rank's heads / FFN
    p.add_argument("--kv-channels", type=int, default=None)
    p.add_argument("--ffn-hidden-size", type=int, default=None)
    p.add_argument("--emulate-tp", type=int, default=0,
                   help="(1 process) time one rank of a TP group of this size: sharded shapes, sequence "
                        "parallelism, ring-chunk GEMMs, collectives as local stand-ins (comm/loopback.py)")
    p.add_argument("--emulate-first-stage", action="store_true",
                   help="(pp = 1 emulation) no LM head: the model outputs hidden states, as pipeline stage 0")
    p.add_argument("--emulate-last-stage", action="store_true",
                   help="(pp = 1 emulation) no embedding: the model takes a received [s/tp, mbs, h] "
                        "activation (random, requires grad) as its input, as the last pipeline stage")
    p.add_argument("--pp-last-layers", type=int, default=None,
                   help="layers on the last pipeline stage (default: balanced against the LM head + CE)")
    p.add_argument("--pp-schedule", choices=["1f1b", "zb", "zbh1", "zbh2"], default="zbh2",
                   help="pipeline schedule (train/schedules.py): 1F1B, or its zero-bubble split backward "
                        "(zbh2: twice the in-flight micro-batches, the lowest simulated bubble at N = 8)")
    p.add_argument("--vpp", type=int, default=1,
                   help="virtual pipeline chunks per rank (interleaved 1F1B; uniform layer split)")
    p.add_argument("--phase-probe", type=int, default=0,
                   help="(pp = 1) after the timed steps, time this many micro-batches as F / B / W: forward, "
                        "backward with the weight-gradient GEMMs held, then those GEMMs "
                        "(train/pipeline_sim.py inputs); reported as fbw_ms")
    p.add_argument("--hidden-dropout", type=float, default=0.1)
    p.add_argument("--attention-dropout", type=float, default=0.1)  # Megatron default (reference run)
    p.add_argument("--zero", type=int, default=1, help="ZeRO-1/2 distributed optimizer when DP > 1")
    p.add_argument("--overlap-grad-reduce", type=int, default=1,
                   help="DP bucket reductions during backward and ZeRO parameter all-gathers during the next "
                        "forward (0: both synchronous; one-GPU Gloo rehearsals)")
    p.add_argument("--overlap-optimizer", type=int, default=0,
                   help="one DP rank: the fused Adam of each gradient bucket on a side stream, overlapped "
                        "with the next step's forward (DistributedDataParallel.overlap_optimizer)")
    p.add_argument("--bucket-size", type=int, default=None,
                   help="DDP bucket elements (default: auto, 8-32 MB from a start-up link timing)")
    p.add_argument("--comm-stats", type=int, default=1, help="phase_ms / per-collective stats in the JSON")
    p.add_argument("--no-flash", action="store_true")
    p.add_argument("--recompute", choices=["none", "full"], default="none")
    p.add_argument("--profile-steps", type=int, default=0)
    p.add_argument("--graph", type=int, default=0,
                   help="capture one whole training step (every micro-batch's forward / backward, the "
                        "gradient sync, the fused Adam with a device-side step count) in a HIP graph after "
                        "the warm-up and replay it: fresh tokens are copied into static buffers and the lr "
                        "set before each replay; dropout masks advance through the device RNG counter "
                        "(ops/functional.enable_graph_rng). pp = 1 (one process per stage emulation too)")
    p.add_argument("--tunableop", type=int, default=1,
                   help="autotune torch's hipBLASLt GEMMs per shape during the (untimed) warmup")
    p.add_argument("--tune-ms", type=int, default=40)
    p.add_argument("--tune-out", type=str, default=None)
    return p.parse_args()


TUNED_GEMMS = os.environ.get("SMDT_TUNED_GEMMS") or os.path.join(
    os.path.dirname(os.path.abspath(__file__)), "profiles", "tunableop", "gfx950_gpt345m_results.csv")
# hipBLASLt algorithm indices of the fused fp32-accumulate wgrad GEMMs, tuned over every algorithm
# hipBLASLt ships for the problem type (SMDT_WGRAD_TUNE=full) on MI355X; reused as-is so the
# selection does not vary run to run.
WGRAD_CACHE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "tunableop",
                           "wgrad_gfx950.csv")
if os.path.exists(WGRAD_CACHE):
    os.environ.setdefault("SMDT_WGRAD_CACHE", WGRAD_CACHE)


def model_label(a, vocab):
    """The BASELINE config's name for the default shape; the explicit shape for any other."""
    shape = f"{a.num_layers}L h{a.hidden_size} {a.num_attention_heads}A, vocab {vocab}"
    if ((a.num_layers, a.hidden_size, a.num_attention_heads, a.seq_length) == (24, 1024, 16, 1024)
            and a.kv_channels in (None, 64) and a.ffn_hidden_size in (None, 4096)):
        return f"gpt2-345m ({shape})"
    known = {(12, 768, 12): "gpt2-small", (32, 4096, 32): "gpt3-6.7b"}
    return f"{known.get((a.num_layers, a.hidden_size, a.num_attention_heads), 'gpt')} ({shape}, seq {a.seq_length})"


def _mlp_fusion_desc():
    """How the MLP's bias + GeLU runs (recorded in the JSON): inside the hand-written GEMMs
    (gemm_tn.hip epilogues, TP = 1) or as the separate bias_act kernels."""
    from smdt_amd.parallel import tensor_parallel as tpm
    if not tpm._FUSED_BIAS_GELU:
        return "bias_act kernels"
    return "gemm_tn epilogues (fc1 bias+GeLU fwd, fc2 dgrad+GeLU bwd)"


def enable_gemm_tuning(a, rank):
    """PyTorch TunableOp over torch's hipBLASLt / rocBLAS GEMMs.

    --tunableop 1 (default): load the per-shape winners measured on MI355X and committed under
    profiles/tunableop/ (no tuning at run time); tune on first use only if that file is absent.
    --tunableop 2: re-tune every shape (minutes) and write the results to --tune-out.
    --tunableop 3: load the committed winners and tune only the shapes missing from them; the
                   table (loaded + new rows) is written to --tune-out at exit (merge it into
                   profiles/tunableop/ with scripts/merge_tunableop.py).
    --tunableop 0: library heuristics only.
    """
    if not (a.tunableop and torch.cuda.is_available()):
        return "off"
    try:
        import tempfile
        import torch.cuda.tunable as tun
        tun.enable(True)
        if a.tunableop == 1 and os.path.exists(TUNED_GEMMS):
            tun.tuning_enable(False)
            tun.set_filename(os.path.join(tempfile.gettempdir(), f"smdt_tunableop_unused_r{rank}.csv"))
            ok = tun.read_file(TUNED_GEMMS)
            return "preloaded" if ok is not False else "preload-failed"
        tun.tuning_enable(True)
        tun.set_max_tuning_duration(a.tune_ms)
        out = a.tune_out or os.path.join(tempfile.gettempdir(), "smdt_tunableop_r%d.csv")
        tun.set_filename(out % rank if "%d" in out else out)
        if a.tunableop == 3 and os.path.exists(TUNED_GEMMS):
            tun.read_file(TUNED_GEMMS)
        return "tuning"
    except Exception as e:  # pragma: no cover
        print(f"[bench] TunableOp unavailable: {e!r}", file=sys.stderr)
        return "unavailable"


HEAD_SPEEDUP = 1.4


def balanced_last_stage_layers(num_layers, pp, h, s, vocab):
    """Transformer layers on the last pipeline stage so that it — which also runs the LM head and
    the cross-entropy — costs what every other stage does. Per token, a layer costs
    72 h^2 (1 + s / 6h) FLOPs (fwd + bwd) and the head 6 V h (Megatron's formula), i.e.
    V / (12 h (1 + s / 6h)) layers' worth of FLOPs (3.5 for GPT-2 345M). The head's three big
    GEMMs run ``HEAD_SPEEDUP`` times faster per FLOP than a layer's mix of attention, small GEMMs
    and elementwise kernels (measured on MI355X at the tp2pp2 rank shape: 14 layers 219 ms,
    10 layers + head 197 ms, profiles/r3_predict/), so the head weighs r = 3.5 / 1.4 = 2.5 layers.
    The last stage gets (L - (pp - 1) r) / pp layers, rounded so the other stages split the rest
    evenly: 13 | 11 for GPT-2 345M at pp = 2."""
    r = vocab / (12.0 * h * (1.0 + s / (6.0 * h))) / HEAD_SPEEDUP
    want = (num_layers - (pp - 1) * r) / pp
    best = None
    for n in range(1, num_layers - pp + 2):
        if (num_layers - n) % (pp - 1):
            continue
        cost = max(n + r, (num_layers - n) / (pp - 1))
        if best is None or cost < best[0] - 1e-9 or (abs(cost - best[0]) < 1e-9 and abs(n - want) < abs(best[1] - want)):
            best = (cost, n)
    return best[1]


# N -> (tp, pp); dp = N / (tp pp)
LAYOUTS = {
    "baseline": {1: (1, 1), 2: (1, 1), 4: (1, 1), 8: (2, 2)},
    "tp": {1: (1, 1), 2: (2, 1), 4: (2, 2), 8: (2, 2)},
    "dp": {},
}


def choose_layout(a, world):
    """(tp, pp, sp, micro_batch, grad_accum) for ``world`` GPUs (see the module docstring)."""
    tp, pp = LAYOUTS[a.layout].get(world, (1, 1))
    tp = a.tp if a.tp is not None else tp
    pp = a.pp if a.pp is not None else pp
    if world % (tp * pp):
        raise SystemExit(f"[bench] world {world} is not divisible by tp {tp} x pp {pp}")
    sp = bool(a.sequence_parallel) if a.sequence_parallel is not None else tp > 1
    replica = a.seqs_per_gpu * tp * pp          # sequences per DP replica per step
    if a.micro_batch_size is not None:
        mbs = a.micro_batch_size
    elif pp == 1:
        mbs = min(replica, 64)
    else:
        # >= 4 pp micro-batches (bubble <= 20 %), at most 32 sequences each: at N = 8 (256
        # sequences per replica) 8 micro-batches of 32 measured 213 ms per rank incl. the 1F1B
        # bubble vs 220 ms for 16 of 16 (benchmarks/predict_mbs.py, profiles/r3_predict/)
        mbs = max(1, min(32, replica // (4 * pp)))
    ga = a.grad_accum if a.grad_accum is not None else max(1, replica // mbs)
    return tp, pp, sp, mbs, ga


def main():
    a = parse()
    if os.environ.get("SMDT_BENCH_DUMP_AFTER"):   # diagnostics: every thread's stack after N s
        import faulthandler
        faulthandler.dump_traceback_later(float(os.environ["SMDT_BENCH_DUMP_AFTER"]), repeat=True)
    from smdt_amd.comm import buckets as comm_buckets
    from smdt_amd.comm import stats as comm_stats
    comm_stats.enable(bool(a.comm_stats))   # before the process group: RCCL per-work timing
    # SMDT_BENCH_BACKEND=gloo: rehearsal of the N > 1 code paths with every rank on ONE GPU (RCCL
    # refuses two ranks on one device); the driver's runs use RCCL
    rank, local, world, backend = init_distributed(os.environ.get("SMDT_BENCH_BACKEND", "nccl"))
    from smdt_amd.utils.debug import collective_log_from_env
    collective_log_from_env()      # SMDT_COLLECTIVE_LOG=<prefix>: per-rank collective issue order
    if world != a.gpus and rank == 0:
        print(f"[bench] note: --gpus {a.gpus} but WORLD_SIZE {world}; using WORLD_SIZE", file=sys.stderr)
    n = world
    if a.emulate_tp:
        if world != 1:
            raise SystemExit("[bench] --emulate-tp runs in one process")
        a.tp, a.pp = 1, 1
        _, _, _, a.micro_batch_size, a.grad_accum = choose_layout(a, world)
        a.tp, sp = a.emulate_tp, a.sequence_parallel is None or bool(a.sequence_parallel)
        st = ps.initialize_emulated_tensor_parallel(a.tp)
    else:
        a.tp, a.pp, sp, a.micro_batch_size, a.grad_accum = choose_layout(a, world)
        st = ps.initialize_model_parallel(a.tp, a.pp, a.vpp if (a.vpp > 1 and a.pp > 1) else None)
    if a.tp > 1:
        # TP exchange overlap of the N = 8 layouts (profiles/r6_fill2/: measured under the paced
        # link stand-in): queued W GEMMs fill the ring-exchange waits, and ring-chunk GEMMs issued
        # beside an in-flight transfer run on gemm_tn with the CUs the transfer leaves.
        # SMDT_W_FILL=0 / SMDT_RING_GEMM_TN=0 turn them off.
        from smdt_amd.parallel import tensor_parallel as _tpm
        _tpm.W_FILL = os.environ.get("SMDT_W_FILL", "1") == "1"
        _tpm._RING_GEMM_TN = os.environ.get("SMDT_RING_GEMM_TN", "1") == "1"
    model_parallel_seed(1234)
    tuned = enable_gemm_tuning(a, rank)
    dev = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")
    vocab = pad_vocab_size(a.vocab_size, 128, a.tp)
    vpp = a.vpp if (a.vpp > 1 and a.pp > 1) else 1
    last_layers = a.pp_last_layers
    if last_layers is None and a.pp > 1 and vpp == 1:
        last_layers = balanced_last_stage_layers(a.num_layers, a.pp, a.hidden_size, a.seq_length, vocab)
    cfg = TransformerConfig(num_layers=a.num_layers, hidden_size=a.hidden_size,
                            num_attention_heads=a.num_attention_heads, max_position_embeddings=a.seq_length,
                            padded_vocab_size=vocab, hidden_dropout=a.hidden_dropout,
                            kv_channels=a.kv_channels, ffn_hidden_size=a.ffn_hidden_size,
                            decoder_last_pipeline_num_layers=last_layers,
                            attention_dropout=a.attention_dropout, params_dtype=torch.bfloat16,
                            sequence_parallel=sp and a.tp > 1, use_flash_attn=not a.no_flash,
                            recompute_granularity="full" if a.recompute == "full" else None,
                            recompute_method="uniform" if a.recompute == "full" else None)
    if vpp > 1:   # interleaved: vpp chunks per rank in one flat DDP buffer (train/training.get_model)
        chunks = []
        for c in range(vpp):
            st.virtual_pp_rank = c
            chunks.append(GPTModel(cfg, pre_process=st.is_first_stage(), post_process=st.is_last_stage(), device=dev))
        st.virtual_pp_rank = 0
        model = torch.nn.ModuleList(chunks)
    else:
        if a.emulate_first_stage and a.emulate_last_stage:
            raise SystemExit("[bench] --emulate-first-stage and --emulate-last-stage exclude each other")
        model = GPTModel(cfg, pre_process=st.is_first_stage() and not a.emulate_last_stage,
                         post_process=st.is_last_stage() and not a.emulate_first_stage, device=dev)
    zero = bool(a.zero) and (st.dp > 1 or (bool(a.overlap_optimizer) and st.pp == 1))
    ddp = DistributedDataParallel(model, bucket_size=a.bucket_size, use_distributed_optimizer=zero,
                                  overlap_param_gather=zero and st.dp > 1 and bool(a.overlap_grad_reduce),
                                  overlap_grad_reduce=bool(a.overlap_grad_reduce))
    use_graph = bool(a.graph) and dev.type == "cuda" and st.pp == 1
    # the xGMI DP engine stays in the captured step (replay-safe; health checked between replays)
    ddp.xgmi_in_graph = use_graph and ddp.xgmi is not None
    opt = MixedPrecisionAdam(ddp, lr=1.5e-4, betas=(0.9, 0.95), eps=1e-8, weight_decay=0.01, clip_grad=1.0,
                             capturable=use_graph)
    if use_graph:
        from smdt_amd.ops import functional as _SF
        _SF.enable_graph_rng(dev)
    sched = OptimizerParamScheduler(opt, max_lr=1.5e-4, min_lr=1e-5, lr_warmup_steps=10, lr_decay_steps=10000,
                                    lr_decay_style="cosine")
    mbs, S = a.micro_batch_size, a.seq_length
    gen = torch.Generator(device=dev)
    gen.manual_seed(1000 + st.dp_rank)

    def batches():
        while True:
            yield torch.randint(0, a.vocab_size, (mbs, S + 1), device=dev, generator=gen)

    it = batches()
    pos = None   # positions 0 .. S-1 in every sequence (the model's broadcast position-table slice)
    # graph mode: the step reads its micro-batches from static buffers refilled before each replay
    static_tok = [torch.empty((mbs, S + 1), dtype=torch.long, device=dev) for _ in range(a.grad_accum)] \
        if use_graph else None
    static_act = None

    def refill():
        for t in static_tok:
            t.copy_(next(it))
        if static_act is not None:
            static_act.normal_(generator=gen)

    def static_batches():
        while True:
            yield from static_tok

    def forward_step(data_iter, m):
        toks = next(data_iter)
        tokens, labels = toks[:, :-1], toks[:, 1:]
        if a.emulate_last_stage:   # the activation a last stage receives from its predecessor
            act = static_act if static_act is not None else \
                torch.randn(shape, device=dev, dtype=torch.bfloat16, generator=gen)
            model.set_input_tensor(act.detach().requires_grad_())
        out = m(tokens, pos, None, labels=labels)

        def loss_func(o):
            loss = o.float().mean()
            return loss, {"lm loss": loss.detach()}
        return out, loss_func

    configure_p2p(overlap=True)   # pipeline receives are waited for at their consumer
    set_pipeline_schedule(a.pp_schedule)
    fb = get_forward_backward_func()
    shape = (S // a.tp if cfg.sequence_parallel else S, mbs, cfg.hidden_size)

    def train_step(stats=False, data=None, lr=None):
        if stats:
            comm_stats.begin_step()
        ddp.zero_grad_buffer()
        # an emulated pipeline stage issues each micro-batch's W GEMMs as its schedule would
        losses = fb(forward_step, data if data is not None else it, ddp, a.grad_accum, tensor_shape=shape,
                    dtype=torch.bfloat16,
                    split_backward=bool(a.emulate_tp) and a.pp_schedule in ("zb", "zbh1", "zbh2"))
        comm_stats.mark("fwd_bwd")
        ddp.finish_grad_sync()
        allreduce_word_embedding_grads(model)   # tied embedding: first + last pipeline stage
        comm_stats.mark("grad_sync")
        opt.step(sched.step(1) if lr is None else None)
        comm_stats.mark("optimizer")
        comm_stats.end_step()
        if use_graph:
            _SF.advance_graph_rng()
        return losses

    graph = None

    def graph_step():
        """Refill the static inputs, set this step's lr (the captured Adam reads it from the
        device), replay. With the xGMI engine inside the graph, its health check runs between
        replays; after a fallback to RCCL the step runs eager from then on."""
        nonlocal graph
        if ddp.xgmi_in_graph and not ddp.health_between_replays():
            graph = None
            return train_step()
        refill()
        opt.set_lr(sched.step(1))
        graph[0].replay()
        return graph[1]

    tw = time.perf_counter()
    for i in range(a.warmup):
        train_step()
        if rank == 0:  # progress line per warmup step (first-use GEMM tuning can take minutes)
            print(f"[bench] warmup step {i + 1}/{a.warmup} done at {time.perf_counter() - tw:.1f}s",
                  file=sys.stderr, flush=True)
    if rank == 0:
        print(f"[bench] warmup ({a.warmup} steps, incl. GEMM autotune) took {time.perf_counter() - tw:.1f}s",
              file=sys.stderr, flush=True)
    graph_note = None
    if use_graph:
        if a.emulate_last_stage:
            static_act = torch.empty(shape, device=dev, dtype=torch.bfloat16)
        refill()
        torch.cuda.synchronize()
        try:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                glosses = train_step(data=static_batches(), lr=False)
            graph = (g, glosses)
            for _ in range(2):
                graph_step()
            graph_note = "captured"
        except Exception as e:  # noqa: BLE001 - report and run eager
            graph_note = f"capture failed, eager: {type(e).__name__}: {str(e)[:160]}"
            print(f"[bench] {graph_note}", file=sys.stderr, flush=True)
            graph = None
        torch.cuda.synchronize()
    run_step = (lambda stats=False: graph_step()) if graph is not None else train_step
    if dist.is_initialized():
        dist.barrier()
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    last = None
    # on GPUs the stats are recorded on two extra steps after the timed ones (below); the host-clock
    # stats of a CPU (Gloo) run cost nothing measurable and are recorded on the timed steps
    cpu_stats = bool(a.comm_stats) and not torch.cuda.is_available()
    for _ in range(a.steps):
        last = run_step(stats=cpu_stats)
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    if dist.is_initialized():
        dist.barrier()
    el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
    if dist.is_initialized():
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    elapsed = float(el.item())
    ms_step = 1000 * elapsed / a.steps
    # phase_ms / comm come from two extra steps after the timed ones: the per-collective events
    # and phase marks cost ~3 % of a step at the N = 8 rank's ~4 k launches per step (207.6 vs
    # 201.8 ms, profiles/r4_comm_stats_cost/), so the timed steps run without them
    if a.comm_stats and not cpu_stats:
        for _ in range(2):
            train_step(stats=True)
        torch.cuda.synchronize()
    explain = comm_stats.summary(ms_step) if a.comm_stats else None
    phases_all = None
    if explain is not None and dist.is_initialized() and world > 1:
        phases_all = [None] * world
        dist.all_gather_object(phases_all, (st.pp_rank, explain["phase_ms"]))
    fbw = probe_fbw(a, ddp, forward_step, it, dev) if (a.phase_probe and st.pp == 1) else None
    from smdt_amd.comm import xgmi
    relay.check_all()            # (after the timed region) no TP-pair exchange timed out
    global_batch = mbs * a.grad_accum * st.dp
    tokens_per_step = global_batch * S
    tps = tokens_per_step * a.steps / elapsed
    fpt = gpt_flops_per_token(cfg, S, recompute=False)
    ref_tps = REF_TFLOPS_PER_GPU * n / fpt
    # the loss lives on the last pipeline stage: share it so rank 0 can report it
    lv = torch.zeros(1, dtype=torch.float32, device=dev)
    if last:
        lv[0] = torch.stack([d["lm loss"] for d in last]).float().mean()
    if dist.is_initialized() and st.pp > 1:
        dist.all_reduce(lv, op=dist.ReduceOp.MAX)
    loss_val = float(lv.item())
    if rank == 0:
        emulated = bool(a.emulate_tp or a.emulate_first_stage or a.emulate_last_stage)
        label = model_label(a, vocab)
        if emulated:
            # ONE rank of a larger job on one GPU, collectives as local copies: its time is an
            # input to benchmarks/predict_scaling.py, never a job throughput (no value / vs_baseline
            # / model TFLOP/s from the whole-model formula)
            head = {"metric": "emulated rank ms/step", "value": round(ms_step, 3), "unit": "ms",
                    "n_gpus": n, "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(ms_step, 3),
                    "higher_is_better": False, "scaling": None, "vs_baseline": None}
        else:
            head = {"metric": ("tokens/sec (whole node) GPT-2 345M pretrain" if label.startswith("gpt2-345m")
                               else f"tokens/sec (whole node) {label.split(' (')[0]} pretrain"),
                    "value": round(tps, 1), "unit": "tokens/s", "n_gpus": n, "steps": a.steps,
                    "warmup": a.warmup, "ms_per_step": round(ms_step, 3), "higher_is_better": True,
                    "scaling": "weak", "vs_baseline": round(tps / ref_tps, 3)}
        rec = {
            **head,
            "dtype": "bf16",
            "data": "synthetic (random tokens, CodeParrot-shaped [mbs, 1025] int64; random-init weights)",
            "config": {"model": label, "global_batch": global_batch,
                       "seq_len": S, "micro_batch": mbs, "grad_accum": a.grad_accum,
                       "parallelism": f"tp{a.tp}pp{a.pp}dp{st.dp}" + ("+sp" if cfg.sequence_parallel else "")
                       + ("+zero1" if zero else "") + (" (one emulated TP rank)" if a.emulate_tp else ""),
                       "layout": a.layout, "tp": a.tp, "pp": a.pp, "dp": st.dp,
                       "pp_layers": ([(a.num_layers - last_layers) // (a.pp - 1)] * (a.pp - 1) + [last_layers]
                                     if (a.pp > 1 and vpp == 1) else [a.num_layers // a.pp] * a.pp),
                       "pp_schedule": (f"interleaved vpp{vpp}" if vpp > 1 else a.pp_schedule) if a.pp > 1 else None,
                       "ddp_bucket": {"elements": ddp.bucket_size, "count": len(ddp.buckets),
                                      **comm_buckets.TUNED},
                       "scaling_note": f"weak: {a.seqs_per_gpu} seqs x {S} tokens per GPU per step",
                       "flash_attn": not a.no_flash, "hidden_dropout": a.hidden_dropout,
                       "attention_dropout": a.attention_dropout, "recompute": a.recompute,
                       "gemm_autotune": tuned,
                       "comm_stream_priority": comm_streams.describe()["comm_stream_priority"],
                       "optimizer_overlap": bool(getattr(ddp, "overlap_optimizer", False)),
                       "mlp_gelu_fusion": _mlp_fusion_desc(),
                       "hip_graph": graph_note,
                       **({"tp_overlap": {"w_fill": _tp_flag("W_FILL"), "ring_gemm_tn": _tp_flag("_RING_GEMM_TN"),
                                          "exchange_cu_reserve": _tp_flag("_CU_RESERVE_ON")}} if a.tp > 1 else {}),
                       **({"link_standin": {"GBps": link_standin()[0], "workgroups": link_standin()[1],
                                            "exchanges_per_step": _split_stats().get("standin_exchanges", 0)}}
                          if emulated and link_standin() else {}),
                       **({"sp_subbatch": 2} if _subbatch_on() else {})},
            **({} if emulated else {
                "model_tflops_per_gpu": round(tps * fpt / n / 1e12, 2),
                "baseline": "41 model-TFLOP/s/GPU (reference GPT-2-small, 16xA100, BASELINE.md) at equal model FLOPs"}),
            "final_loss": loss_val,
        }
        comm = {**relay.TUNED, **xgmi.TUNED}
        if comm:  # run-time RCCL-vs-kernel decisions on this node (comm/relay.py, comm/xgmi.py)
            rec["comm_tuning"] = comm
        if fbw is not None:
            rec["fbw_ms"] = fbw
        if explain is not None:
            rec["phase_ms"] = _mean_phases([p for _, p in phases_all]) if phases_all else explain["phase_ms"]
            if phases_all and st.pp > 1:
                rec["phase_ms_by_pp_stage"] = {
                    str(k): _mean_phases([p for r, p in phases_all if r == k]) for k in range(st.pp)}
            rec["comm"] = explain["comm"]   # rank 0's collectives, per step
        print(json.dumps(rec), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()


def _tp_flag(name):
    from smdt_amd.parallel import tensor_parallel as _tp
    return bool(getattr(_tp, name))


def _split_stats():
    from smdt_amd.parallel import tensor_parallel as _tp
    return _tp.SPLIT_STATS


def _subbatch_on():
    from smdt_amd.models import transformer as _T
    return _T._SUBBATCH == 2


def probe_fbw(a, ddp, forward_step, it, dev):
    """Untimed diagnostics after the timed steps: per micro-batch, the forward (F), the backward
    with the deferred weight-gradient queue held (B: the input-gradient chain a pipeline stage must
    finish before it sends) and the flush of that queue (W), each bracketed by device events
    (median over ``a.phase_probe`` micro-batches). Gradients accumulate into the buffers and are
    zeroed at the end; nothing here is part of the measured step."""
    from smdt_amd.parallel.tensor_parallel import DEFERRED_WGRAD
    cuda = dev.type == "cuda"

    def stamp():
        if cuda:
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            return e
        return time.perf_counter()

    def ms(t0, t1):
        return t0.elapsed_time(t1) if cuda else 1e3 * (t1 - t0)
    rows = []
    ddp.set_sync_enabled(False)
    for _ in range(a.phase_probe):
        t0 = stamp()
        out, loss_func = forward_step(it, ddp)
        loss, _ = loss_func(out)
        t1 = stamp()
        DEFERRED_WGRAD.defer = True
        try:
            loss.backward()
        finally:
            DEFERRED_WGRAD.defer = False
        t2 = stamp()
        DEFERRED_WGRAD.flush()
        t3 = stamp()
        if cuda:
            torch.cuda.synchronize()
        rows.append((ms(t0, t1), ms(t1, t2), ms(t2, t3)))
    ddp.set_sync_enabled(True)
    ddp.zero_grad_buffer()

    def med(i):
        v = sorted(r[i] for r in rows)
        return round(v[len(v) // 2], 3)
    return {"F": med(0), "B": med(1), "W": med(2), "micro_batches": len(rows)}


def _mean_phases(ps_):
    keys = ps_[0].keys()
    return {k: round(sum(p[k] for p in ps_) / len(ps_), 3) for k in keys}


if __name__ == "__main__":
    main()
