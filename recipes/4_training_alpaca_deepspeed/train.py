"""Alpaca supervised fine-tuning on MI355X (recipe 4; reference
/root/reference/4_training_alpaca_deepspeed/train.py).

Same CLI and flow as the reference script — HF-style ``(ModelArguments, DataArguments,
TrainingArguments)`` flags, ``--deepspeed <json>`` with "auto" values, special-token handling +
embedding resize, Alpaca prompt formatting with prompt-masked labels, ``Trainer.train()``,
``save_state()``, ``save_model()`` — on the smdt_amd stack: HIP kernels (flash attention, fused
LN/RMSNorm+residual, SwiGLU/ReLU, fused CE), ZeRO over RCCL, fused AdamW.

Launch (one process per GPU)::

    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 train.py \
        --model_name_or_path facebook/opt-125m --data_path alpaca_data.json --bf16 True \
        --output_dir out --num_train_epochs 1 --per_device_train_batch_size 4 \
        --gradient_accumulation_steps 8 --learning_rate 2e-5 --warmup_ratio 0.03 \
        --deepspeed configs/default_offload_opt_param.json

Offline: a model name without local files builds the architecture with random init; a missing
``--data_path`` file is replaced by a synthetic Alpaca-shaped JSON (``--synthetic_examples``).
"""
import os
import sys

# SageMaker MPI launch -> torch env (reference train.py:21-25); torchrun envs pass through.
if "OMPI_COMM_WORLD_RANK" in os.environ and "RANK" not in os.environ:
    os.environ["LOCAL_RANK"] = os.environ["OMPI_COMM_WORLD_LOCAL_RANK"]
    os.environ["RANK"] = os.environ["OMPI_COMM_WORLD_RANK"]
    os.environ["WORLD_SIZE"] = os.environ["OMPI_COMM_WORLD_SIZE"]
    os.environ["NODE_RANK"] = str(int(os.environ["RANK"]) // 8)

_HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.abspath(os.path.join(_HERE, "..", "..")))

from dataclasses import dataclass, field  # noqa: E402

import torch  # noqa: E402

from smdt_amd.data import sft  # noqa: E402
from smdt_amd.models.hf import HFCausalLM  # noqa: E402
from smdt_amd.parallel import zero_init  # noqa: E402
from smdt_amd.train import hf_args  # noqa: E402
from smdt_amd.train.sft_trainer import Trainer, setup_distributed  # noqa: E402
from smdt_amd.train.zero import load_ds_config  # noqa: E402


@dataclass
class ModelArguments(hf_args.ModelArguments):
    pass


@dataclass
class DataArguments(hf_args.DataArguments):
    synthetic_examples: int = field(default=52002, metadata={"help": "examples to generate if data_path is missing"})


@dataclass
class TrainingArguments(hf_args.TrainingArguments):
    cache_dir: str = field(default=None)
    optim: str = field(default="adamw_torch")
    model_max_length: int = field(default=512, metadata={"help": "Maximum sequence length (right padded / truncated)."})


def smart_tokenizer_and_embedding_resize(special_tokens_dict, tokenizer, model: HFCausalLM):
    """Add special tokens, grow the vocab, and initialise the new rows with the mean of the old
    ones (input and output embeddings) — reference train.py:92-112. Rows are addressed by vocab
    index (the table itself is padded to a multiple of 128 for the GEMM tiles)."""
    old = model.vocab_size
    num_new = tokenizer.add_special_tokens(special_tokens_dict)
    model.resize_token_embeddings(len(tokenizer))
    if num_new > 0:
        new = len(tokenizer)
        with torch.no_grad():
            w_in = model.get_input_embeddings().weight
            w_in[old:new] = w_in[:old].float().mean(0, keepdim=True).to(w_in.dtype)
            w_out = model.get_output_embeddings().weight
            if w_out is not w_in:
                w_out[old:new] = w_out[:old].float().mean(0, keepdim=True).to(w_out.dtype)


def train():
    parser = hf_args.ArgumentParser((ModelArguments, DataArguments, TrainingArguments))
    model_args, data_args, training_args = parser.parse_args_into_dataclasses()
    rank, local, world, device = setup_distributed(training_args)

    dtype = torch.bfloat16 if training_args.bf16 else torch.float16 if training_args.fp16 else torch.float32
    # ZeRO-3: every rank keeps only its shard of each parameter from the moment it is built
    # (DeepSpeed zero.Init; parallel/zero_init.py)
    stage = int(load_ds_config(training_args.deepspeed).get("zero_optimization", {}).get("stage", 0))
    with zero_init.Init(enabled=stage >= 3 and world > 1) as zi:
        model = HFCausalLM.from_pretrained(model_args.model_name_or_path, params_dtype=dtype, device=device,
                                           cache_dir=training_args.cache_dir)
    if zi.params and rank == 0:
        print(f"[zero.Init] {zi.params} parameters partitioned at construction over {zi.dp} ranks: "
              f"{zi.shard_bytes / 1e6:.1f} MB of shards per rank (peak {zi.peak_bytes / 1e6:.1f} MB)", flush=True)
    tokenizer = sft.load_tokenizer(model_args.model_name_or_path, cache_dir=training_args.cache_dir,
                                   model_max_length=training_args.model_max_length,
                                   model_type=model.hf_config.get("model_type"))
    special = {}
    if tokenizer.pad_token is None:
        special["pad_token"] = sft.DEFAULT_PAD_TOKEN
    if tokenizer.eos_token is None:
        special["eos_token"] = sft.DEFAULT_EOS_TOKEN
    if tokenizer.bos_token is None:
        special["bos_token"] = sft.DEFAULT_BOS_TOKEN
    if tokenizer.unk_token is None:
        special["unk_token"] = sft.DEFAULT_UNK_TOKEN
    with zero_init.gathered([model.get_input_embeddings().weight, model.get_output_embeddings().weight]):
        smart_tokenizer_and_embedding_resize(special, tokenizer, model)

    if not data_args.data_path or not os.path.exists(data_args.data_path):
        path = data_args.data_path or os.path.join(training_args.output_dir, "synthetic_alpaca.json")
        if rank == 0:
            print(f"[alpaca] {path} not found: writing {data_args.synthetic_examples} synthetic examples", flush=True)
            sft.write_synthetic_alpaca(path, data_args.synthetic_examples)
        if world > 1:
            torch.distributed.barrier()
        data_args.data_path = path
    cache = training_args.cache_dir or os.path.join(training_args.output_dir, ".sft_cache")
    if local == 0:  # tokenise once per node into the shared cache, then everyone memory-loads it
        sft.SupervisedDataset(data_args.data_path, tokenizer, cache_dir=cache)
    if world > 1:
        torch.distributed.barrier()
    data_module = sft.make_supervised_data_module(tokenizer, data_args, cache_dir=cache,
                                                  pad_to_multiple_of=training_args.pad_to_multiple_of)
    trainer = Trainer(model=model, tokenizer=tokenizer, args=training_args, **data_module)
    trainer.train()
    trainer.save_state()
    trainer.save_model(output_dir=training_args.output_dir)


if __name__ == "__main__":
    train()
