"""Pretrain GPT on MI355X (entry point compatible with the reference recipe).

Same contract as /root/reference/3_training_megatron-lm/pretrain_gpt.py: the
launcher passes Megatron flags verbatim (e.g. ``--num-layers 12 ... --fp16 true``), ranks come
from the OMPI_COMM_WORLD_* / torchrun environment, and the same four hooks feed
``pretrain(...)``: ``model_provider``, ``get_batch`` (TP-rank-0 read + broadcast),
``loss_func`` (masked mean + DP-averaged logging loss) and ``forward_step``.

MI355X-specific: ``CUDA_DEVICE_MAX_CONNECTIONS=1`` has no HIP meaning; ordering of the async TP
collectives against compute is guaranteed by issuing them on RCCL's stream from the same host
thread (see smdt_amd.parallel.tensor_parallel), so nothing needs to be exported here.
"""
import os
import sys
from functools import partial

# Make the in-tree framework importable when run from the recipe folder (source_dir layout).
_HERE = os.path.dirname(os.path.abspath(__file__))
for _cand in (os.path.join(_HERE, "..", ".."), os.environ.get("SMDT_ROOT", "")):
    if _cand and os.path.isdir(os.path.join(_cand, "smdt_amd")) and _cand not in sys.path:
        sys.path.insert(0, os.path.abspath(_cand))

from smdt_amd.comm import bridge_ompi_env  # noqa: E402

bridge_ompi_env()  # OMPI_COMM_WORLD_* -> RANK / LOCAL_RANK / WORLD_SIZE / NODE_RANK

import torch  # noqa: E402

from smdt_amd.comm import print_rank_0  # noqa: E402
from smdt_amd.data.gpt_dataset import build_train_valid_test_datasets  # noqa: E402
from smdt_amd.models.gpt import GPTModel  # noqa: E402
from smdt_amd.parallel import state as ps  # noqa: E402
from smdt_amd.parallel import tensor_parallel  # noqa: E402
from smdt_amd.train.arguments import core_transformer_config_from_args, get_args, get_timers, get_tokenizer  # noqa: E402
from smdt_amd.train.training import ModelType, pretrain  # noqa: E402
from smdt_amd.train.utils import (average_losses_across_data_parallel_group, context_parallel_slice,  # noqa: E402
                                  get_ltor_masks_and_position_ids)


def model_provider(pre_process=True, post_process=True):
    """Build the model."""
    print_rank_0("building GPT model ...")
    config = core_transformer_config_from_args(get_args())
    dev = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else None
    return GPTModel(config, pre_process=pre_process, post_process=post_process, parallel_output=True, device=dev)


def get_batch(data_iterator):
    """Read on TP rank 0, broadcast to the TP group, shift into tokens / labels."""
    args = get_args()
    tokenizer = get_tokenizer()
    data = next(data_iterator) if data_iterator is not None else None
    if data is not None and torch.cuda.is_available():
        data = {k: v.cuda(non_blocking=True) for k, v in data.items()}
    b = tensor_parallel.broadcast_data(["text"], data, torch.int64)
    tokens_ = b["text"].long()
    labels = tokens_[:, 1:].contiguous()
    tokens = tokens_[:, :-1].contiguous()
    need_mask = args.reset_attention_mask or not args.use_flash_attn
    attention_mask, loss_mask, position_ids = get_ltor_masks_and_position_ids(
        tokens, tokenizer.eod, args.reset_position_ids, args.reset_attention_mask, args.eod_mask_loss,
        build_attention_mask=need_mask)
    # --context-parallel-size: this rank keeps its contiguous chunk of the sequence
    tokens, labels, loss_mask, position_ids = context_parallel_slice(tokens, labels, loss_mask, position_ids)
    return tokens, labels, loss_mask, attention_mask, position_ids


def loss_func(loss_mask, output_tensor):
    losses = output_tensor.float()
    loss_mask = loss_mask.view(-1).float()
    loss = torch.sum(losses.view(-1) * loss_mask) / loss_mask.sum()
    averaged_loss = average_losses_across_data_parallel_group([loss])
    return loss, {"lm loss": averaged_loss[0]}


def forward_step(data_iterator, model):
    """Forward step."""
    timers = get_timers()
    timers("batch-generator", log_level=2).start()
    tokens, labels, loss_mask, attention_mask, position_ids = get_batch(data_iterator)
    timers("batch-generator").stop()
    # the loss mask tells the fused LM head + CE the reduction loss_func applies
    output_tensor = model(tokens, position_ids, attention_mask, labels=labels, loss_mask=loss_mask)
    return output_tensor, partial(loss_func, loss_mask)


def train_valid_test_datasets_provider(train_val_test_num_samples):
    """Build train, valid, and test datasets."""
    args = get_args()
    print_rank_0("> building train, validation, and test datasets for GPT ...")
    train_ds, valid_ds, test_ds = build_train_valid_test_datasets(
        data_prefix=args.data_path, data_impl=args.data_impl, splits_string=args.split,
        train_valid_test_num_samples=train_val_test_num_samples, seq_length=args.seq_length, seed=args.seed,
        skip_warmup=(not args.mmap_warmup), train_data_prefix=args.train_data_path,
        valid_data_prefix=args.valid_data_path, test_data_prefix=args.test_data_path,
        data_cache_path=args.data_cache_path)
    print_rank_0("> finished creating GPT datasets ...")
    return train_ds, valid_ds, test_ds


if __name__ == "__main__":
    pretrain(train_valid_test_datasets_provider, model_provider, ModelType.encoder_or_decoder, forward_step,
             args_defaults={"tokenizer_type": "GPT2BPETokenizer"})
