"""Learning-rate / weight-decay schedules.

``OptimizerParamScheduler`` mirrors Megatron's (`--lr-warmup-iters`,
`--lr-decay-iters`, `--lr-decay-style {constant,linear,cosine,inverse-square-root}`, `--min-lr`,
`--start/end-weight-decay`, `--weight-decay-incr-style`, `--override-opt_param-scheduler`,
`--use-checkpoint-opt_param-scheduler`: /root/reference/3_training_megatron-lm/megatron/
arguments.py:684-714, :876-919). ``WarmupDecayLR`` is DeepSpeed's schedule used by the Alpaca
recipe (`default_offload_opt_param.json:15-22`), ``StepLR`` the MNIST one.
"""
from __future__ import annotations

import math


class OptimizerParamScheduler:
    def __init__(self, optimizer, max_lr, min_lr, lr_warmup_steps, lr_decay_steps, lr_decay_style="linear",
                 start_wd=0.0, end_wd=0.0, wd_incr_steps=1, wd_incr_style="constant",
                 use_checkpoint_opt_param_scheduler=True, override_opt_param_scheduler=False):
        self.optimizer = optimizer
        self.max_lr, self.min_lr = float(max_lr), float(min_lr)
        assert self.min_lr >= 0.0 and self.max_lr >= self.min_lr
        self.lr_warmup_steps = int(lr_warmup_steps)
        self.lr_decay_steps = max(int(lr_decay_steps), 1)
        assert self.lr_warmup_steps < self.lr_decay_steps or self.lr_decay_steps == 1
        self.lr_decay_style = lr_decay_style
        self.start_wd, self.end_wd = float(start_wd), float(end_wd)
        self.wd_incr_steps, self.wd_incr_style = max(int(wd_incr_steps), 1), wd_incr_style
        self.use_ckpt = use_checkpoint_opt_param_scheduler
        self.override = override_opt_param_scheduler
        self.num_steps = 0
        self.step(0)

    def get_wd(self):
        if self.num_steps > self.wd_incr_steps:
            return self.end_wd
        if self.wd_incr_style == "constant":
            return self.end_wd
        ratio = self.num_steps / self.wd_incr_steps
        delta = self.end_wd - self.start_wd
        if self.wd_incr_style == "linear":
            coeff = ratio
        elif self.wd_incr_style == "cosine":
            coeff = 0.5 * (math.cos(math.pi * (1 - ratio)) + 1.0)
        else:
            raise ValueError(self.wd_incr_style)
        return self.start_wd + coeff * delta

    def get_lr(self):
        n = self.num_steps
        if self.lr_warmup_steps > 0 and n <= self.lr_warmup_steps:
            return self.max_lr * n / self.lr_warmup_steps
        if self.lr_decay_style == "constant":
            return self.max_lr
        if n > self.lr_decay_steps:
            return self.min_lr
        if self.lr_decay_style == "inverse-square-root":
            w = max(self.lr_warmup_steps, 1)
            return max(self.min_lr, self.max_lr * math.sqrt(w) / math.sqrt(max(n, 1)))
        ratio = (n - self.lr_warmup_steps) / max(self.lr_decay_steps - self.lr_warmup_steps, 1)
        delta = self.max_lr - self.min_lr
        if self.lr_decay_style == "linear":
            coeff = 1.0 - ratio
        elif self.lr_decay_style == "cosine":
            coeff = 0.5 * (math.cos(math.pi * ratio) + 1.0)
        else:
            raise ValueError(self.lr_decay_style)
        return self.min_lr + coeff * delta

    def step(self, increment=1):
        self.num_steps += increment
        lr, wd = self.get_lr(), self.get_wd()
        opt = self.optimizer
        if hasattr(opt, "lr"):
            opt.lr = lr
        if hasattr(opt, "weight_decay") and self.wd_incr_style != "constant":
            opt.weight_decay = wd
        for g in getattr(opt, "param_groups", []):
            g["lr"] = lr
        return lr

    def state_dict(self):
        return {"max_lr": self.max_lr, "min_lr": self.min_lr, "lr_warmup_steps": self.lr_warmup_steps,
                "lr_decay_steps": self.lr_decay_steps, "lr_decay_style": self.lr_decay_style,
                "num_steps": self.num_steps, "start_wd": self.start_wd, "end_wd": self.end_wd}

    def load_state_dict(self, d):
        if not self.override and self.use_ckpt:
            for k in ("max_lr", "min_lr", "lr_warmup_steps", "lr_decay_steps", "lr_decay_style", "start_wd", "end_wd"):
                if k in d:
                    setattr(self, k, d[k])
        self.num_steps = 0
        self.step(int(d.get("num_steps", 0)))


class WarmupDecayLR:
    """DeepSpeed WarmupDecayLR: linear (or log) warmup from warmup_min_lr to warmup_max_lr over
    warmup_num_steps, then linear decay to 0 at total_num_steps."""

    def __init__(self, optimizer, total_num_steps, warmup_min_lr=0.0, warmup_max_lr=1e-3, warmup_num_steps=1000,
                 warmup_type="log"):
        self.optimizer = optimizer
        self.total = int(total_num_steps)
        self.min_lr, self.max_lr = float(warmup_min_lr), float(warmup_max_lr)
        self.warm = max(int(warmup_num_steps), 2)  # DeepSpeed clamps to 2 (log warmup divides by log(warm))
        self.warmup_type = warmup_type
        self.last = -1
        self.step()

    def get_lr(self, n):
        if n < self.warm:
            if self.warmup_type == "log":
                g = math.log(n + 1) / math.log(self.warm)
            else:
                g = n / self.warm
            return self.min_lr + (self.max_lr - self.min_lr) * g
        return self.max_lr * max(0.0, (self.total - n) / max(1.0, self.total - self.warm))

    def step(self):
        self.last += 1
        lr = self.get_lr(self.last)
        if hasattr(self.optimizer, "lr"):
            self.optimizer.lr = lr
        for g in getattr(self.optimizer, "param_groups", []):
            g["lr"] = lr
        return lr

    def get_last_lr(self):
        return [self.get_lr(self.last)]

    def state_dict(self):
        return {"last": self.last}

    def load_state_dict(self, d):
        self.last = int(d["last"]) - 1
        self.step()


class LambdaWarmupScheduler:
    """HF ``get_scheduler`` equivalents (``--lr_scheduler_type``): linear / cosine / constant /
    constant_with_warmup / polynomial(power 1) with ``num_warmup_steps`` linear warmup from 0."""

    def __init__(self, optimizer, kind: str, base_lr: float, num_warmup_steps: int, num_training_steps: int,
                 min_lr_ratio: float = 0.0):
        self.optimizer = optimizer
        self.kind = kind
        self.base_lr = float(base_lr)
        self.warm = int(num_warmup_steps)
        self.total = max(int(num_training_steps), 1)
        self.min_ratio = min_lr_ratio
        self.last = -1
        self.step()

    def factor(self, n):
        if n < self.warm:
            return n / max(1, self.warm)
        if self.kind in ("constant", "constant_with_warmup"):
            return 1.0
        prog = (n - self.warm) / max(1, self.total - self.warm)
        if self.kind == "cosine":
            return max(0.0, 0.5 * (1.0 + math.cos(math.pi * prog)))
        return max(self.min_ratio, 1.0 - prog)      # linear / polynomial

    def get_lr(self, n):
        return self.base_lr * self.factor(n)

    def step(self):
        self.last += 1
        lr = self.get_lr(self.last)
        if hasattr(self.optimizer, "lr"):
            self.optimizer.lr = lr
        for g in getattr(self.optimizer, "param_groups", []):
            g["lr"] = lr
        return lr

    def get_last_lr(self):
        return [self.get_lr(self.last)]

    def state_dict(self):
        return {"last": self.last}

    def load_state_dict(self, d):
        self.last = int(d["last"]) - 1
        self.step()
