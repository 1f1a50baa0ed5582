"""Megatron-compatible command line (flag names verbatim) + validation + TransformerConfig bridge.

Front-end parity with /root/reference/3_training_megatron-lm/megatron/arguments.py (SURVEY R9,
§5.6): the recipe's hyperparameters dict (NB3:399-428) is serialised by the launcher into
``--num-layers 12 --fp16 true ...`` and must parse unchanged. Notable semantics kept:
  * ``--fp16`` takes a string bool (the reference's local revision, arguments.py:964);
  * ``validate_args`` derives the DP size, global batch, micro-batch count, params dtype,
    enforces SP only with TP > 1, distributed optimizer only with local DDP, etc.;
  * ``args_defaults`` fill values the user did not pass (e.g. tokenizer_type);
  * deprecated flags (``--batch-size``, ``--warmup``, ``--model-parallel-size``,
    ``--checkpoint-activations``) are rejected with the same advice.

Flags that only matter on NVIDIA stacks (``--transformer-impl``, fp8) are accepted and
ignored; table-driven groups keep the list easy to audit against the reference.
"""
from __future__ import annotations

import argparse
import os
from typing import Optional

import torch

from ..models.transformer import TransformerConfig


def str_bool(s) -> bool:
    return str(s).lower() in ("true", "t", "yes", "1", "y")


# (flag, kwargs) per group. dest is derived by argparse (dashes -> underscores).
_GROUPS = {
    "network size": [
        ("--num-layers", dict(type=int, default=None)),
        ("--encoder-num-layers", dict(type=int, default=None)),
        ("--decoder-num-layers", dict(type=int, default=None)),
        ("--hidden-size", dict(type=int, default=None)),
        ("--ffn-hidden-size", dict(type=int, default=None)),
        ("--num-attention-heads", dict(type=int, default=None)),
        ("--kv-channels", dict(type=int, default=None)),
        ("--group-query-attention", dict(action="store_true")),
        ("--num-query-groups", dict(type=int, default=1)),
        ("--max-position-embeddings", dict(type=int, default=None)),
        ("--position-embedding-type", dict(type=str, default="learned_absolute", choices=["learned_absolute", "rope"])),
        ("--use-rotary-position-embeddings", dict(action="store_true")),
        ("--rotary-percent", dict(type=float, default=1.0)),
        ("--no-position-embedding", dict(action="store_false", dest="add_position_embedding")),
        ("--make-vocab-size-divisible-by", dict(type=int, default=128)),
        ("--layernorm-epsilon", dict(type=float, default=1e-5)),
        ("--normalization", dict(type=str, default="LayerNorm", choices=["LayerNorm", "RMSNorm"])),
        ("--apply-layernorm-1p", dict(action="store_true")),
        ("--apply-residual-connection-post-layernorm", dict(action="store_true")),
        ("--openai-gelu", dict(action="store_true")),
        ("--squared-relu", dict(action="store_true")),
        ("--swiglu", dict(action="store_true")),
        ("--onnx-safe", dict(type=str_bool, default=None)),
        ("--bert-no-binary-head", dict(action="store_false", dest="bert_binary_head")),
        ("--num-experts", dict(type=int, default=None)),
        ("--untie-embeddings-and-output-weights", dict(action="store_true")),
        ("--embedding-weights-in-fp32", dict(action="store_true")),
    ],
    "logging": [
        ("--log-params-norm", dict(action="store_true")),
        ("--log-num-zeros-in-grad", dict(action="store_true")),
        ("--timing-log-level", dict(type=int, default=0, choices=range(0, 3))),
        ("--no-barrier-with-level-1-timing", dict(action="store_false", dest="barrier_with_L1_time")),
        ("--timing-log-option", dict(type=str, default="minmax", choices=["max", "minmax", "all"])),
        ("--tensorboard-log-interval", dict(type=int, default=1)),
        ("--tensorboard-queue-size", dict(type=int, default=1000)),
        ("--log-timers-to-tensorboard", dict(action="store_true")),
        ("--log-batch-size-to-tensorboard", dict(action="store_true")),
        ("--no-log-learnig-rate-to-tensorboard", dict(action="store_false", dest="log_learning_rate_to_tensorboard")),
        ("--no-log-loss-scale-to-tensorboard", dict(action="store_false", dest="log_loss_scale_to_tensorboard")),
        ("--log-validation-ppl-to-tensorboard", dict(action="store_true")),
        ("--log-memory-to-tensorboard", dict(action="store_true")),
        ("--log-world-size-to-tensorboard", dict(action="store_true")),
        ("--metrics-jsonl", dict(type=str, default=None)),
    ],
    "regularization": [
        ("--attention-dropout", dict(type=float, default=0.1)),
        ("--hidden-dropout", dict(type=float, default=0.1)),
        ("--weight-decay", dict(type=float, default=0.01)),
        ("--start-weight-decay", dict(type=float, default=None)),
        ("--end-weight-decay", dict(type=float, default=None)),
        ("--weight-decay-incr-style", dict(type=str, default="constant", choices=["constant", "linear", "cosine"])),
        ("--clip-grad", dict(type=float, default=1.0)),
        ("--adam-beta1", dict(type=float, default=0.9)),
        ("--adam-beta2", dict(type=float, default=0.999)),
        ("--adam-eps", dict(type=float, default=1e-08)),
        ("--sgd-momentum", dict(type=float, default=0.9)),
    ],
    "training": [
        ("--micro-batch-size", dict(type=int, default=None)),
        ("--batch-size", dict(type=int, default=None)),
        ("--global-batch-size", dict(type=int, default=None)),
        ("--rampup-batch-size", dict(nargs="*", default=None)),
        ("--recompute-activations", dict(action="store_true")),
        ("--recompute-granularity", dict(type=str, default=None, choices=["full", "selective"])),
        ("--distribute-saved-activations", dict(action="store_true")),
        ("--recompute-method", dict(type=str, default=None, choices=["uniform", "block"])),
        ("--recompute-num-layers", dict(type=int, default=1)),
        ("--profile", dict(action="store_true")),
        ("--profile-step-start", dict(type=int, default=10)),
        ("--profile-step-end", dict(type=int, default=12)),
        ("--profile-ranks", dict(nargs="+", type=int, default=[0])),
        ("--checkpoint-activations", dict(action="store_true")),
        ("--train-iters", dict(type=int, default=None)),
        ("--train-samples", dict(type=int, default=None)),
        ("--log-interval", dict(type=int, default=100)),
        ("--exit-interval", dict(type=int, default=None)),
        ("--exit-duration-in-mins", dict(type=int, default=None)),
        ("--exit-signal-handler", dict(action="store_true")),
        ("--tensorboard-dir", dict(type=str, default=None)),
        ("--no-masked-softmax-fusion", dict(action="store_false", dest="masked_softmax_fusion")),
        ("--no-bias-gelu-fusion", dict(action="store_false", dest="bias_gelu_fusion")),
        ("--no-bias-dropout-fusion", dict(action="store_false", dest="bias_dropout_fusion")),
        ("--use-flash-attn", dict(action="store_true")),
        ("--no-flash-attn", dict(action="store_true", help="force the unfused softmax path")),
        ("--disable-bias-linear", dict(action="store_false", dest="add_bias_linear")),
        ("--optimizer", dict(type=str, default="adam", choices=["adam", "sgd"])),
        ("--dataloader-type", dict(type=str, default=None, choices=["single", "cyclic"])),
        ("--no-async-tensor-model-parallel-allreduce", dict(action="store_false", dest="async_tensor_model_parallel_allreduce")),
        ("--no-persist-layer-norm", dict(action="store_true")),
        ("--sequence-parallel", dict(action="store_true")),
        ("--no-gradient-accumulation-fusion", dict(action="store_false", dest="gradient_accumulation_fusion")),
    ],
    "initialization": [
        ("--seed", dict(type=int, default=1234)),
        ("--data-parallel-random-init", dict(action="store_true")),
        ("--init-method-std", dict(type=float, default=0.02)),
        ("--init-method-xavier-uniform", dict(action="store_true")),
    ],
    "learning rate": [
        ("--lr", dict(type=float, default=None)),
        ("--lr-decay-style", dict(type=str, default="linear", choices=["constant", "linear", "cosine", "inverse-square-root"])),
        ("--lr-decay-iters", dict(type=int, default=None)),
        ("--lr-decay-samples", dict(type=int, default=None)),
        ("--lr-warmup-fraction", dict(type=float, default=None)),
        ("--lr-warmup-iters", dict(type=int, default=0)),
        ("--lr-warmup-samples", dict(type=int, default=0)),
        ("--warmup", dict(type=int, default=None)),
        ("--min-lr", dict(type=float, default=0.0)),
        ("--override-opt_param-scheduler", dict(action="store_true")),
        ("--use-checkpoint-opt_param-scheduler", dict(action="store_true")),
    ],
    "checkpointing": [
        ("--save", dict(type=str, default=None)),
        ("--async-save", dict(action="store_true")),   # Megatron-core: write checkpoints in the background
        ("--save-interval", dict(type=int, default=None)),
        ("--no-save-optim", dict(action="store_true", default=None)),
        ("--no-save-rng", dict(action="store_true", default=None)),
        ("--load", dict(type=str, default=None)),
        ("--no-load-optim", dict(action="store_true", default=None)),
        ("--no-load-rng", dict(action="store_true", default=None)),
        ("--finetune", dict(action="store_true")),
        ("--no-initialization", dict(action="store_false", dest="perform_initialization")),
        ("--use-checkpoint-args", dict(action="store_true")),
        ("--exit-on-missing-checkpoint", dict(action="store_true")),
    ],
    "mixed precision": [
        ("--fp16", dict(type=str_bool, default=False)),   # string bool: reference revision
        ("--bf16", dict(type=str_bool, nargs="?", const=True, default=False)),
        ("--loss-scale", dict(type=float, default=None)),
        ("--initial-loss-scale", dict(type=float, default=2 ** 32)),
        ("--min-loss-scale", dict(type=float, default=1.0)),
        ("--loss-scale-window", dict(type=float, default=1000)),
        ("--hysteresis", dict(type=int, default=2)),
        ("--fp32-residual-connection", dict(action="store_true")),
        ("--no-query-key-layer-scaling", dict(action="store_false", dest="apply_query_key_layer_scaling")),
        ("--attention-softmax-in-fp32", dict(action="store_true")),
        ("--accumulate-allreduce-grads-in-fp32", dict(action="store_true")),
        ("--fp16-lm-cross-entropy", dict(action="store_true")),
    ],
    "distributed": [
        ("--tensor-model-parallel-size", dict(type=int, default=1)),
        # Megatron-core's flag; Ulysses all-to-all context parallelism (parallel/context_parallel.py)
        ("--context-parallel-size", dict(type=int, default=1)),
        ("--pipeline-model-parallel-size", dict(type=int, default=1)),
        ("--pipeline-model-parallel-split-rank", dict(type=int, default=None)),
        ("--model-parallel-size", dict(type=int, default=None)),
        ("--num-layers-per-virtual-pipeline-stage", dict(type=int, default=None)),
        ("--overlap-p2p-communication", dict(action="store_true")),
        # non-interleaved pipeline schedule (train/schedules.py): Megatron's 1F1B by default; the
        # zero-bubble split backward forms hold up to pp micro-batches of W operands in HBM
        ("--pp-schedule", dict(default="1f1b", choices=["1f1b", "zb", "zbh1", "zbh2"])),
        ("--overlap-param-gather", dict(action="store_true")),
        ("--distributed-backend", dict(default="nccl", choices=["nccl", "gloo", "smddp", "rccl"])),
        ("--distributed-timeout-minutes", dict(type=int, default=10)),
        ("--DDP-impl", dict(default="local", choices=["local", "torch"])),
        ("--no-contiguous-buffers-in-local-ddp", dict(action="store_false", dest="use_contiguous_buffers_in_local_ddp")),
        ("--no-scatter-gather-tensors-in-pipeline", dict(action="store_false", dest="scatter_gather_tensors_in_pipeline")),
        ("--use-ring-exchange-p2p", dict(action="store_true")),
        ("--local_rank", dict(type=int, default=None)),
        ("--lazy-mpu-init", dict(type=str_bool, default=None)),
        ("--use-cpu-initialization", dict(action="store_true", default=None)),
        ("--empty-unused-memory-level", dict(default=0, type=int, choices=[0, 1, 2])),
        ("--standalone-embedding-stage", dict(action="store_true")),
        ("--decoder-first-pipeline-num-layers", dict(type=int, default=None)),
        ("--decoder-last-pipeline-num-layers", dict(type=int, default=None)),
        ("--use-distributed-optimizer", dict(action="store_true")),
        ("--ddp-bucket-size", dict(type=int, default=None)),  # None: auto (comm/buckets.py)
    ],
    "validation": [
        ("--eval-iters", dict(type=int, default=100)),
        ("--eval-interval", dict(type=int, default=1000)),
        ("--skip-train", dict(action="store_true")),
    ],
    "data and dataloader": [
        ("--data-path", dict(nargs="*", default=None)),
        ("--split", dict(type=str, default="969, 30, 1")),
        ("--train-data-path", dict(nargs="*", default=None)),
        ("--valid-data-path", dict(nargs="*", default=None)),
        ("--test-data-path", dict(nargs="*", default=None)),
        ("--data-cache-path", dict(default=None)),
        ("--vocab-size", dict(type=int, default=None)),
        ("--vocab-file", dict(type=str, default=None)),
        ("--merge-file", dict(type=str, default=None)),
        ("--vocab-extra-ids", dict(type=int, default=0)),
        ("--seq-length", dict(type=int, default=None)),
        ("--encoder-seq-length", dict(type=int, default=None)),
        ("--decoder-seq-length", dict(type=int, default=None)),
        ("--retriever-seq-length", dict(type=int, default=256)),
        ("--sample-rate", dict(type=float, default=1.0)),
        ("--mask-prob", dict(type=float, default=0.15)),
        ("--short-seq-prob", dict(type=float, default=0.1)),
        ("--mmap-warmup", dict(action="store_true")),
        ("--num-workers", dict(type=int, default=2)),
        ("--tokenizer-type", dict(type=str, default=None,
                                  choices=["BertWordPieceLowerCase", "BertWordPieceCase", "GPT2BPETokenizer",
                                           "SentencePieceTokenizer", "GPTSentencePieceTokenizer",
                                           "HuggingFaceTokenizer", "NullTokenizer"])),
        ("--tokenizer-model", dict(type=str, default=None)),
        ("--data-impl", dict(type=str, default="infer", choices=["mmap", "infer", "lazy", "cached"])),
        ("--reset-position-ids", dict(action="store_true")),
        ("--reset-attention-mask", dict(action="store_true")),
        ("--eod-mask-loss", dict(action="store_true")),
        ("--mock-data", dict(action="store_true", help="synthetic tokens instead of --data-path")),
    ],
    "autoresume": [
        ("--adlr-autoresume", dict(action="store_true")),
        ("--adlr-autoresume-interval", dict(type=int, default=1000)),
    ],
    "transformer-engine": [
        ("--fp8-e4m3", dict(action="store_true")),
        ("--fp8-hybrid", dict(action="store_true")),
        ("--no-fp8-wgrad", dict(action="store_false", dest="fp8_wgrad")),
        ("--fp8-margin", dict(type=int, default=0)),
        ("--fp8-interval", dict(type=int, default=1)),
        ("--transformer-impl", dict(default="local", choices=["local", "transformer_engine"])),
        ("--fp8-amax-history-len", dict(type=int, default=1)),
        ("--fp8-amax-compute-algo", dict(default="most_recent", choices=["most_recent", "max"])),
    ],
    # Task families of the reference's Megatron tree that this framework does not train (vision
    # classification / inpainting / DINO, ICT / REALM biencoder retrieval, Retro, text-generation
    # inference): accepted so a reference hyperparameter dict parses unchanged, and ignored with a
    # warning when set to a non-default value (validate_args). Reference:
    # 3_training_megatron-lm/megatron/arguments.py:478-483 (inference), 500-503 (Bert embedder),
    # 1182-1199 (Retro), 1239-1305 (biencoder, vision).
    "inference (accepted, ignored)": [
        ("--inference-batch-times-seqlen-threshold", dict(type=int, default=512)),
        ("--max-tokens-to-oom", dict(type=int, default=12000)),
        ("--output-bert-embeddings", dict(action="store_true")),
        ("--bert-embedder-type", dict(default="megatron", choices=["megatron", "huggingface"])),
    ],
    "retro (accepted, ignored)": [
        ("--retro-workdir", dict(default=None)),
        ("--retro-add-retriever", dict(action="store_true", default=False)),
        ("--retro-cyclic-train-iters", dict(type=int, default=None)),
        ("--retro-encoder-layers", dict(type=int, default=2)),
        ("--retro-encoder-hidden-dropout", dict(type=float, default=0.1)),
        ("--retro-encoder-attention-dropout", dict(type=float, default=0.1)),
        ("--retro-num-neighbors", dict(type=int, default=2)),
        ("--retro-num-retrieved-chunks", dict(type=int, default=2)),
        ("--retro-return-doc-ids", dict(action="store_true")),
    ],
    "biencoder (accepted, ignored)": [
        ("--ict-head-size", dict(type=int, default=None)),
        ("--biencoder-projection-dim", dict(type=int, default=0)),
        ("--biencoder-shared-query-context-model", dict(action="store_true")),
        ("--ict-load", dict(type=str, default=None)),
        ("--bert-load", dict(type=str, default=None)),
        ("--titles-data-path", dict(type=str, default=None)),
        ("--query-in-block-prob", dict(type=float, default=0.1)),
        ("--use-one-sent-docs", dict(action="store_true")),
        ("--evidence-data-path", dict(type=str, default=None)),
        ("--retriever-report-topk-accuracies", dict(nargs="+", type=int, default=[])),
        ("--retriever-score-scaling", dict(action="store_true")),
        ("--block-data-path", dict(type=str, default=None)),
        ("--embedding-path", dict(type=str, default=None)),
        ("--indexer-batch-size", dict(type=int, default=128)),
        ("--indexer-log-interval", dict(type=int, default=1000)),
    ],
    "vision (accepted, ignored)": [
        ("--num-classes", dict(type=int, default=1000)),
        ("--img-h", dict(type=int, default=224)),
        ("--img-w", dict(type=int, default=224)),
        ("--num-channels", dict(type=int, default=3)),
        ("--patch-dim", dict(type=int, default=16)),
        ("--classes-fraction", dict(type=float, default=1.0)),
        ("--data-per-class-fraction", dict(type=float, default=1.0)),
        ("--no-data-sharding", dict(action="store_false", dest="data_sharding")),
        ("--head-lr-mult", dict(type=float, default=1.0)),
        ("--vision-pretraining", dict(action="store_true")),
        ("--vision-pretraining-type", dict(type=str, default="classify", choices=["classify", "inpaint", "dino"])),
        ("--vision-backbone-type", dict(type=str, default="vit", choices=["vit", "mit", "swin"])),
        ("--swin-backbone-type", dict(type=str, default="tiny", choices=["tiny", "base", "h3"])),
        ("--mask-type", dict(type=str, default="random", choices=["random", "row"])),
        ("--mask-factor", dict(type=float, default=1.0)),
        ("--iter-per-epoch", dict(type=int, default=1250)),
        ("--dino-local-img-size", dict(type=int, default=96)),
        ("--dino-local-crops-number", dict(type=int, default=10)),
        ("--dino-head-hidden-size", dict(type=int, default=2048)),
        ("--dino-bottleneck-size", dict(type=int, default=256)),
        ("--dino-freeze-last-layer", dict(type=float, default=1)),
        ("--dino-norm-last-layer", dict(action="store_true")),
        ("--dino-warmup-teacher-temp", dict(type=float, default=0.04)),
        ("--dino-teacher-temp", dict(type=float, default=0.07)),
        ("--dino-warmup-teacher-temp-epochs", dict(type=int, default=30)),
    ],
}

# groups whose flags are parsed but drive nothing here (see the comment above)
IGNORED_GROUPS = tuple(t for t in _GROUPS if t.endswith("(accepted, ignored)"))


# Model-form / NVIDIA-stack flags that parse but change nothing here: (flag, (dest, default)).
# validate_args warns when one is set to a non-default value, so a run never silently differs.
_NO_EFFECT = [
    ("--fp32-residual-connection", ("fp32_residual_connection", False)),
    ("--embedding-weights-in-fp32", ("embedding_weights_in_fp32", False)),
    ("--fp16-lm-cross-entropy", ("fp16_lm_cross_entropy", False)),
    ("--transformer-impl", ("transformer_impl", "local")),
    ("--fp8-e4m3", ("fp8_e4m3", False)),
    ("--fp8-hybrid", ("fp8_hybrid", False)),
]


def ignored_flags_set(args) -> list:
    """The accepted-but-ignored flags (IGNORED_GROUPS) whose value differs from the default."""
    out = []
    for title in IGNORED_GROUPS:
        for flag, kw in _GROUPS[title]:
            dest = kw.get("dest", flag.lstrip("-").replace("-", "_"))
            if kw.get("action") == "store_true":
                default = kw.get("default", False)
            elif kw.get("action") == "store_false":
                default = True
            else:
                default = kw.get("default")
            if hasattr(args, dest) and getattr(args, dest) != default:
                out.append(flag)
    return out


def build_parser(extra_args_provider=None) -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(description="smdt_amd Megatron-compatible arguments", allow_abbrev=False)
    for title, flags in _GROUPS.items():
        g = p.add_argument_group(title=title)
        for flag, kw in flags:
            g.add_argument(flag, **kw)
    if extra_args_provider is not None:
        p = extra_args_provider(p)
    return p


def parse_args(extra_args_provider=None, ignore_unknown_args=False, argv=None):
    p = build_parser(extra_args_provider)
    if ignore_unknown_args:
        args, _ = p.parse_known_args(argv)
    else:
        args = p.parse_args(argv)
    args.rank = int(os.environ.get("RANK", os.environ.get("OMPI_COMM_WORLD_RANK", "0")))
    args.world_size = int(os.environ.get("WORLD_SIZE", os.environ.get("OMPI_COMM_WORLD_SIZE", "1")))
    return args


def validate_args(args, defaults=None):
    defaults = defaults or {}
    ignored = ignored_flags_set(args)
    if ignored and int(getattr(args, "rank", 0) or 0) == 0:
        import warnings
        warnings.warn("accepted but ignored (task families this framework does not train: vision, "
                      "biencoder / ICT, Retro, inference): " + " ".join(ignored), stacklevel=2)
    args.tensor_model_parallel_size = min(args.tensor_model_parallel_size, args.world_size)
    assert args.world_size % args.tensor_model_parallel_size == 0, "world size not divisible by TP"
    args.pipeline_model_parallel_size = min(args.pipeline_model_parallel_size,
                                            args.world_size // args.tensor_model_parallel_size)
    mp = args.tensor_model_parallel_size * args.pipeline_model_parallel_size * args.context_parallel_size
    assert args.world_size % mp == 0, "world size not divisible by TP * PP * CP"
    args.data_parallel_size = args.world_size // mp
    if args.rank == 0:
        print(f"using world size: {args.world_size}, data-parallel-size: {args.data_parallel_size}, "
              f"context-parallel size: {args.context_parallel_size}, "
              f"tensor-model-parallel size: {args.tensor_model_parallel_size}, "
              f"pipeline-model-parallel size: {args.pipeline_model_parallel_size} ", flush=True)
    if args.context_parallel_size > 1:
        heads = args.num_attention_heads // args.tensor_model_parallel_size
        assert heads % args.context_parallel_size == 0, \
            "context parallelism re-shards attention heads: (heads / TP) must be divisible by CP"
        assert args.seq_length is None or args.seq_length % args.context_parallel_size == 0, \
            "sequence length must be divisible by the context-parallel size"
    assert args.batch_size is None, "--batch-size argument is no longer valid, use --micro-batch-size instead"
    assert args.warmup is None, "--warmup argument is no longer valid, use --lr-warmup-fraction instead"
    assert args.model_parallel_size is None, "--model-parallel-size is no longer valid, use --tensor-model-parallel-size"
    if args.checkpoint_activations:
        raise SystemExit("--checkpoint-activations is no longer valid, use --recompute-activations, or, for more "
                         "control, --recompute-granularity and --recompute-method.")
    if args.recompute_activations:
        args.recompute_granularity = "selective"
    for k, v in defaults.items():
        if getattr(args, k, None) is None:
            setattr(args, k, v)
        elif args.rank == 0:
            print(f"WARNING: overriding default arguments for {k}:{v} with {k}:{getattr(args, k)}", flush=True)
    assert args.micro_batch_size is not None and args.micro_batch_size > 0
    if args.global_batch_size is None:
        args.global_batch_size = args.micro_batch_size * args.data_parallel_size
    assert args.global_batch_size % (args.micro_batch_size * args.data_parallel_size) == 0, \
        "global batch size must be divisible by micro-batch-size * data-parallel-size"
    args.num_micro_batches = args.global_batch_size // (args.micro_batch_size * args.data_parallel_size)
    if args.rampup_batch_size:
        if len(args.rampup_batch_size) != 3:
            raise ValueError("--rampup-batch-size expects <start batch size> <batch size increment> <ramp-up samples>")
        args.rampup_batch_size = [int(v) for v in args.rampup_batch_size]
        if args.train_iters is not None and args.train_samples is None:
            raise ValueError("--rampup-batch-size needs --train-samples (iteration counts vary while ramping)"
                             " — Megatron's rule")
    if args.num_layers_per_virtual_pipeline_stage is not None:
        # Megatron requires pp > 2 here; the canonical p2p op order (train/schedules.py) makes pp = 2 safe
        assert args.pipeline_model_parallel_size >= 2, "interleaved schedule needs pipeline parallelism"
        assert args.num_layers % args.num_layers_per_virtual_pipeline_stage == 0
        args.virtual_pipeline_model_parallel_size = (args.num_layers // args.pipeline_model_parallel_size //
                                                     args.num_layers_per_virtual_pipeline_stage)
    else:
        args.virtual_pipeline_model_parallel_size = None
    # precision
    args.params_dtype = torch.float32
    if args.fp16:
        assert not args.bf16
        args.params_dtype = torch.half
    if args.bf16:
        args.params_dtype = torch.bfloat16
        args.accumulate_allreduce_grads_in_fp32 = True   # Megatron forces fp32 grads with bf16
    if args.use_distributed_optimizer:
        assert args.DDP_impl == "local", "distributed optimizer requires local DDP"
    # iterations / samples
    if args.train_iters is not None:
        assert args.train_samples is None
        if args.lr_decay_iters is None:
            args.lr_decay_iters = args.train_iters
    if args.lr_warmup_fraction is not None:
        assert args.lr_warmup_iters == 0
    for req in ("num_layers", "hidden_size", "num_attention_heads", "max_position_embeddings"):
        assert getattr(args, req) is not None, f"--{req.replace('_', '-')} is required"
    if args.seq_length is None:
        args.seq_length = args.encoder_seq_length
    assert args.seq_length is not None and args.max_position_embeddings >= args.seq_length
    if args.ffn_hidden_size is None:
        args.ffn_hidden_size = 4 * args.hidden_size if not args.swiglu else int(8 * args.hidden_size / 3)
    if args.kv_channels is None:
        assert args.hidden_size % args.num_attention_heads == 0
        args.kv_channels = args.hidden_size // args.num_attention_heads
    if not args.group_query_attention:
        args.num_query_groups = args.num_attention_heads
    if args.use_rotary_position_embeddings:
        args.position_embedding_type = "rope"
    if not args.add_position_embedding and args.position_embedding_type == "learned_absolute":
        args.position_embedding_type = "none"          # --no-position-embedding: no positional table
    no_effect = [f for f, d in _NO_EFFECT if getattr(args, d[0], d[1]) != d[1]]
    if no_effect and args.rank == 0:
        import warnings
        warnings.warn("accepted but without effect here (the model keeps its standard form): "
                      + " ".join(no_effect), stacklevel=2)
    if args.tensor_model_parallel_size == 1 and args.sequence_parallel:
        if args.rank == 0:
            print("Disabling sequence parallelism because tensor model parallel size is 1", flush=True)
        args.sequence_parallel = False
    if args.sequence_parallel:
        args.async_tensor_model_parallel_allreduce = False
    if args.distribute_saved_activations:
        # Megatron's rules: only with full recompute and without sequence parallelism
        if args.recompute_granularity != "full":
            raise ValueError("--distribute-saved-activations needs --recompute-granularity full")
        if args.sequence_parallel:
            raise ValueError("--distribute-saved-activations cannot be combined with --sequence-parallel")
    for k in ("no_save_optim", "no_save_rng", "no_load_optim", "no_load_rng", "use_cpu_initialization"):
        if getattr(args, k) is None:
            setattr(args, k, False)
    if args.start_weight_decay is None:
        args.start_weight_decay = args.weight_decay
    if args.end_weight_decay is None:
        args.end_weight_decay = args.weight_decay
    # Flash attention is the default on gfx950; --no-flash-attn forces the unfused K1 path.
    args.use_flash_attn = (args.use_flash_attn or not args.no_flash_attn) and not args.no_flash_attn
    return args


def print_args(args):
    if args.rank != 0:
        return
    print("------------------------ arguments ------------------------", flush=True)
    for k in sorted(vars(args)):
        print(f"  {k} {'.' * (48 - len(k))} {getattr(args, k)}", flush=True)
    print("-------------------- end of arguments ---------------------", flush=True)


def core_transformer_config_from_args(args) -> TransformerConfig:
    act = "gelu"
    if args.swiglu:
        act = "swiglu"
    elif args.squared_relu:
        act = "squared_relu"
    elif args.openai_gelu:
        act = "gelu"
    return TransformerConfig(
        num_layers=args.num_layers, hidden_size=args.hidden_size, num_attention_heads=args.num_attention_heads,
        num_query_groups=args.num_query_groups, ffn_hidden_size=args.ffn_hidden_size, kv_channels=args.kv_channels,
        decoder_first_pipeline_num_layers=getattr(args, "decoder_first_pipeline_num_layers", None),
        decoder_last_pipeline_num_layers=getattr(args, "decoder_last_pipeline_num_layers", None),
        hidden_dropout=args.hidden_dropout, attention_dropout=args.attention_dropout,
        layernorm_epsilon=args.layernorm_epsilon, normalization=args.normalization, activation=act,
        add_bias_linear=args.add_bias_linear, position_embedding_type=args.position_embedding_type,
        rotary_percent=args.rotary_percent, max_position_embeddings=args.max_position_embeddings,
        padded_vocab_size=args.padded_vocab_size,
        untie_embeddings_and_output_weights=args.untie_embeddings_and_output_weights,
        init_method_std=args.init_method_std, params_dtype=args.params_dtype, seed=args.seed,
        init_method="xavier_uniform" if args.init_method_xavier_uniform else "normal",
        layernorm_zero_centered_gamma=args.apply_layernorm_1p, num_experts=args.num_experts,
        apply_residual_connection_post_layernorm=args.apply_residual_connection_post_layernorm,
        perform_initialization=args.perform_initialization,
        use_cpu_initialization=bool(args.use_cpu_initialization),
        sequence_parallel=args.sequence_parallel,
        async_tensor_model_parallel_allreduce=args.async_tensor_model_parallel_allreduce,
        masked_softmax_fusion=args.masked_softmax_fusion, bias_gelu_fusion=args.bias_gelu_fusion,
        bias_dropout_fusion=args.bias_dropout_fusion, use_flash_attn=args.use_flash_attn,
        apply_query_key_layer_scaling=args.apply_query_key_layer_scaling,
        recompute_granularity=args.recompute_granularity, recompute_method=args.recompute_method,
        recompute_num_layers=args.recompute_num_layers,
        distribute_saved_activations=bool(args.distribute_saved_activations))


# ------------------------------------------------------------------------ micro-batch calculator (U2)
class MicroBatchCalculator:
    """Megatron's num-microbatches calculator: constant, or ``--rampup-batch-size <start> <incr>
    <ramp samples>`` (/root/reference/3_training_megatron-lm/megatron/arguments.py:734-745): the
    global batch grows from ``start`` by ``incr`` every ramp_samples / ((global - start) / incr)
    consumed samples until it reaches ``--global-batch-size``; micro-batches per step =
    current global batch / (micro batch x data-parallel size)."""

    def __init__(self, global_batch_size: int, micro_batch_size: int, dp: int, rampup=None):
        self.gbs, self.mbs, self.dp = int(global_batch_size), int(micro_batch_size), int(dp)
        self.per = self.mbs * self.dp
        self.rampup = None
        if rampup:
            start, incr, samples = (int(v) for v in rampup)
            if start <= 0 or incr <= 0 or samples < 0:
                raise ValueError(f"--rampup-batch-size values must be positive, got {rampup}")
            diff = self.gbs - start
            if diff < 0 or diff % incr:
                raise ValueError(f"global batch {self.gbs} - start {start} must be a non-negative multiple of {incr}")
            if start % self.per or incr % self.per:
                raise ValueError(f"ramp-up start {start} and increment {incr} must be multiples of micro batch "
                                 f"x dp = {self.per}")
            self.rampup = (start, incr, samples, samples / max(diff // incr, 1))
        self.current = self.gbs if self.rampup is None else self.rampup[0]

    def update(self, consumed_samples: int):
        if self.rampup is not None:
            start, incr, samples, per_incr = self.rampup
            if consumed_samples > samples:
                self.current = self.gbs
            else:
                self.current = min(self.gbs, start + int(consumed_samples / per_incr) * incr)
        return self.current

    @property
    def num_micro_batches(self) -> int:
        return self.current // self.per

    def describe(self) -> str:
        if self.rampup is None:
            return f"setting number of micro-batches to constant {self.num_micro_batches}"
        start, incr, samples, _ = self.rampup
        return (f"will use batch size rampup starting from global batch size {start} to global batch size "
                f"{self.gbs} with batch size increments {incr} over {samples} samples.")


# ------------------------------------------------------------------------ global singletons (U2)
_GLOBAL = {"args": None, "tokenizer": None, "timers": None}


def set_global(name, value):
    _GLOBAL[name] = value


def get_args():
    return _GLOBAL["args"]


def get_tokenizer():
    return _GLOBAL["tokenizer"]


def get_timers():
    return _GLOBAL["timers"]
