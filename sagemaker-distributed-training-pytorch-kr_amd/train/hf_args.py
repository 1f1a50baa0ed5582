"""HF-Trainer-compatible argument dataclasses and parser.

The Alpaca recipe parses ``(ModelArguments, DataArguments, TrainingArguments)`` with
``transformers.HfArgumentParser`` (/root/reference/4_training_alpaca_deepspeed/train.py:72-89,
:210-211) from the SageMaker hyperparameter CLI (NB4:463-485: ``--bf16 False``,
``--deepspeed <json>``, ``--evaluation_strategy no`` ...). ``TrainingArguments`` here keeps the HF
field names and defaults for every flag that recipe (and typical SFT scripts) pass, so the same
command line works; unknown flags are an error like in HF.
"""
from __future__ import annotations

import argparse
import dataclasses
import json
import os
import sys
from dataclasses import dataclass, field
from typing import List, Optional, Tuple, Union, get_args, get_origin, get_type_hints


@dataclass
class ModelArguments:
    model_name_or_path: Optional[str] = field(default="facebook/opt-125m")


@dataclass
class DataArguments:
    data_path: Optional[str] = field(default=None, metadata={"help": "Path to the training data."})


@dataclass
class TrainingArguments:
    output_dir: str = "trainer_output"
    overwrite_output_dir: bool = False
    do_train: bool = False
    do_eval: bool = False
    num_train_epochs: float = 3.0
    max_steps: int = -1
    per_device_train_batch_size: int = 8
    per_device_eval_batch_size: int = 8
    gradient_accumulation_steps: int = 1
    learning_rate: float = 5e-5
    weight_decay: float = 0.0
    adam_beta1: float = 0.9
    adam_beta2: float = 0.999
    adam_epsilon: float = 1e-8
    max_grad_norm: float = 1.0
    lr_scheduler_type: str = "linear"
    warmup_ratio: float = 0.0
    warmup_steps: int = 0
    logging_dir: Optional[str] = None
    logging_strategy: str = "steps"
    logging_first_step: bool = False
    logging_steps: float = 500
    evaluation_strategy: str = "no"
    eval_strategy: Optional[str] = None
    eval_steps: Optional[float] = None
    save_strategy: str = "steps"
    save_steps: float = 500
    save_total_limit: Optional[int] = None
    save_only_model: bool = False
    seed: int = 42
    data_seed: Optional[int] = None
    bf16: bool = False
    fp16: bool = False
    tf32: Optional[bool] = None
    local_rank: int = -1
    dataloader_num_workers: int = 0
    dataloader_drop_last: bool = False
    dataloader_pin_memory: bool = True
    remove_unused_columns: bool = True
    group_by_length: bool = False
    report_to: Optional[List[str]] = None
    run_name: Optional[str] = None
    disable_tqdm: Optional[bool] = None
    deepspeed: Optional[str] = None
    fsdp: Optional[str] = ""
    gradient_checkpointing: bool = False
    resume_from_checkpoint: Optional[str] = None
    optim: str = "adamw_torch"
    ddp_find_unused_parameters: Optional[bool] = None
    ddp_backend: Optional[str] = None
    # stanford_alpaca additions (train.py:82-89)
    cache_dir: Optional[str] = None
    model_max_length: int = 512
    # MI355X additions
    pad_to_multiple_of: int = field(default=128, metadata={"help": "round batch length up (flash-attn tiles)"})
    metrics_jsonl: Optional[str] = None

    def __post_init__(self):
        if self.eval_strategy is not None:
            self.evaluation_strategy = self.eval_strategy
        if isinstance(self.report_to, str):
            self.report_to = [self.report_to]
        if self.report_to is None:
            self.report_to = ["none"]
        if self.logging_dir is None:
            self.logging_dir = os.path.join(self.output_dir, "runs")
        if self.local_rank == -1 and "LOCAL_RANK" in os.environ:
            self.local_rank = int(os.environ["LOCAL_RANK"])
        if self.bf16 and self.fp16:
            raise ValueError("--bf16 and --fp16 are exclusive")

    @property
    def world_size(self) -> int:
        return int(os.environ.get("WORLD_SIZE", "1"))

    @property
    def process_index(self) -> int:
        return int(os.environ.get("RANK", "0"))

    @property
    def train_batch_size(self) -> int:
        return self.per_device_train_batch_size

    def get_warmup_steps(self, num_training_steps: int) -> int:
        import math
        return self.warmup_steps if self.warmup_steps > 0 else math.ceil(num_training_steps * self.warmup_ratio)

    def to_dict(self):
        return dataclasses.asdict(self)

    def to_json_string(self):
        return json.dumps(self.to_dict(), indent=2, sort_keys=True, default=str)


def _str2bool(v):
    if isinstance(v, bool):
        return v
    lv = str(v).lower()
    if lv in ("yes", "true", "t", "y", "1"):
        return True
    if lv in ("no", "false", "f", "n", "0"):
        return False
    raise argparse.ArgumentTypeError(f"truthy value expected, got {v}")


class ArgumentParser(argparse.ArgumentParser):
    """``HfArgumentParser`` equivalent: one ``--field`` per dataclass field, bools accept a bare
    flag or an explicit True/False value (SageMaker passes ``--bf16 False``)."""

    def __init__(self, dataclass_types, **kw):
        kw.setdefault("allow_abbrev", False)
        super().__init__(**kw)
        if dataclasses.is_dataclass(dataclass_types):
            dataclass_types = [dataclass_types]
        self.dataclass_types = list(dataclass_types)
        for dt in self.dataclass_types:
            self._add(dt)

    def _add(self, dt):
        hints = get_type_hints(dt)
        for f in dataclasses.fields(dt):
            if not f.init:
                continue
            t = hints[f.name]
            origin = get_origin(t)
            if origin is Union:
                inner = [a for a in get_args(t) if a is not type(None)]
                t = inner[0] if inner else str
                origin = get_origin(t)
            kw = {"help": f.metadata.get("help", "")}
            default = f.default if f.default is not dataclasses.MISSING else (
                f.default_factory() if f.default_factory is not dataclasses.MISSING else None)
            names = [f"--{f.name}"]
            if "_" in f.name:
                names.append(f"--{f.name.replace('_', '-')}")
            if t is bool:
                kw.update(type=_str2bool, nargs="?", const=True, default=default)
            elif origin in (list, List):
                (it,) = get_args(t) or (str,)
                kw.update(type=it, nargs="+", default=default)
            else:
                kw.update(type=t, default=default)
            self.add_argument(*names, dest=f.name, **kw)

    def parse_args_into_dataclasses(self, args=None, return_remaining_strings=False) -> Tuple:
        if args is None:
            args = sys.argv[1:]
        if len(args) == 1 and args[0].endswith(".json") and os.path.exists(args[0]):
            return self.parse_json_file(args[0])
        ns, rem = self.parse_known_args(args)
        outs = []
        for dt in self.dataclass_types:
            keys = {f.name for f in dataclasses.fields(dt) if f.init}
            outs.append(dt(**{k: v for k, v in vars(ns).items() if k in keys}))
        if rem and not return_remaining_strings:
            raise ValueError(f"Some specified arguments are not used by the ArgumentParser: {rem}")
        return (*outs, rem) if return_remaining_strings else tuple(outs)

    def parse_dict(self, d):
        outs = []
        for dt in self.dataclass_types:
            keys = {f.name for f in dataclasses.fields(dt) if f.init}
            outs.append(dt(**{k: v for k, v in d.items() if k in keys}))
        return tuple(outs)

    def parse_json_file(self, path):
        with open(path) as f:
            return self.parse_dict(json.load(f))
