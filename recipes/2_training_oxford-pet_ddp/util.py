"""Oxford-Pet recipe utilities (same API as /root/reference/2_training_oxford-pet_ddp/util.py).

torch_model / accuracy / save_model / AverageMeter / ProgressMeter / adjust_learning_rate /
save_history / to_python_float / init_modelhistory / checkpoint sync helpers.

Differences (documented, deliberate):
  * ``torch_model`` builds architectures from ``smdt_amd.models`` (no torchvision zoo); with
    ``pretrained=True`` it loads ``$SMDT_PRETRAINED_DIR/<name>.pth`` if present (torchvision
    naming; ``weights_only=True``), otherwise it warns and starts from random init — there is no
    download path;
  * the classifier really is resized to ``num_classes`` (the reference only set an attribute,
    ``model.head.out_features = num_classes``, leaving a 1000-way head, util.py:53-54);
  * the S3 sync helpers become local directory syncs (the job API has no S3).
"""
import json
import logging
import os
import shutil
import sys

import torch
import torch.nn as nn

logger = logging.getLogger(__name__)
logger.setLevel(logging.DEBUG)
logger.addHandler(logging.StreamHandler(sys.stdout))


def torch_model(model_name, num_classes=0, pretrained=True):
    from smdt_amd.models import zoo
    if model_name == "inception_v3":
        raise RuntimeError("Currently, inception_v3 is not supported by this example.")
    model = zoo.create(model_name)
    if pretrained:
        d = os.environ.get("SMDT_PRETRAINED_DIR", "")
        path = os.path.join(d, f"{model_name}.pth") if d else ""
        if path and os.path.exists(path):
            print("=> using pre-trained model '{}'".format(model_name))
            model.load_state_dict(torch.load(path, map_location="cpu", weights_only=True))
        else:
            print("=> pre-trained weights for '{}' not available offline; creating model with random init"
                  .format(model_name))
    else:
        print("=> creating model '{}'".format(model_name))
    if num_classes > 0:
        zoo.reset_classifier(model, num_classes)
    return model


def accuracy(output, target, topk=(1,)):
    """Top-k precision (percent) of ``output`` logits [N, C] against ``target`` [N], one 1-element
    tensor per k. One ``topk`` call for the largest k; a hit at rank j counts for every k > j."""
    with torch.no_grad():
        kmax = max(topk)
        idx = output.topk(kmax, dim=1, largest=True, sorted=True).indices          # [N, kmax]
        hit_at = (idx == target.unsqueeze(1)).float()                               # [N, kmax]
        cum = hit_at.cumsum(dim=1).clamp_(max=1.0).sum(dim=0)                       # hits within top-j
        scale = 100.0 / max(target.numel(), 1)
        return [cum[k - 1:k] * scale for k in topk]


def save_model(state, is_best, args):
    """Write ``state`` to <model_dir>/checkpoint.pth (temp file + rename, so a crash never leaves
    a truncated checkpoint) and mirror it to model_best.pth when ``is_best``."""
    logger.info("Saving the model.")
    os.makedirs(args.model_dir, exist_ok=True)
    target = os.path.join(args.model_dir, "checkpoint.pth")
    tmp = target + ".part"
    torch.save(state, tmp)
    os.replace(tmp, target)
    if is_best:
        shutil.copy2(target, os.path.join(args.model_dir, "model_best.pth"))


class AverageMeter:
    """Running value / count-weighted mean of a metric; ``str()`` renders "name val (avg)" with the
    format spec ``fmt`` (e.g. ":6.3f")."""

    def __init__(self, name, fmt=":f"):
        self.name, self.fmt = name, fmt
        self.reset()

    def reset(self):
        self.val, self.sum, self.count = 0, 0, 0

    @property
    def avg(self):
        return self.sum / self.count if self.count else 0

    def update(self, val, n=1):
        """Record ``val`` as the mean of ``n`` samples."""
        self.val = val
        self.sum, self.count = self.sum + val * n, self.count + n

    def __str__(self):
        spec = self.fmt[1:] if self.fmt.startswith(":") else self.fmt
        return f"{self.name} {format(self.val, spec)} ({format(self.avg, spec)})"


class ProgressMeter:
    """Prints "<prefix>[ batch/total]" followed by every meter, tab separated."""

    def __init__(self, num_batches, meters, prefix=""):
        self.total = int(num_batches)
        self.width = len(str(self.total))
        self.meters = list(meters)
        self.prefix = prefix

    def display(self, batch):
        head = f"{self.prefix}[{batch:{self.width}d}/{self.total:{self.width}d}]"
        print("\t".join([head] + [str(m) for m in self.meters]))


def adjust_learning_rate(optimizer, epoch, step, len_epoch, args):
    """Step decay — one x0.1 per 30 epochs plus an extra one from epoch 80 — with a per-step linear
    warm-up over the first 5 epochs, written into every param group."""
    decays = epoch // 30 + int(epoch >= 80)
    lr = args.lr * 0.1 ** decays
    if epoch < 5:
        lr *= (epoch * len_epoch + step + 1) / (5 * len_epoch)
    if args.rank == 0:
        print(f"epoch = {epoch}, step = {step}, lr = {lr}")
    for group in optimizer.param_groups:
        group["lr"] = lr


def save_history(path, history):
    """JSON dump of {metric: [floats]} (tensors / numpy scalars converted)."""
    plain = {name: [float(x) for x in values] for name, values in history.items()}
    with open(path, "w", encoding="utf-8") as f:
        f.write(json.dumps(plain, sort_keys=True, indent=4, separators=(",", ":")))


def to_python_float(t):
    """A Python number from a 0-d / 1-element tensor, a sequence, or a number."""
    item = getattr(t, "item", None)
    if callable(item):
        return item()
    if isinstance(t, (list, tuple)):
        return t[0]
    return t


def init_modelhistory(model_history):
    for k in ("epoch", "batch_idx", "batch_time", "losses", "top1", "top5", "val_epoch", "val_batch_idx",
              "val_batch_time", "val_losses", "val_top1", "val_top5", "val_avg_epoch", "val_avg_batch_time",
              "val_avg_losses", "val_avg_top1", "val_avg_top5"):
        model_history[k] = []
    return model_history


def sync_local_checkpoints_to_store(local_path="/opt/ml/checkpoints", store_path=None):
    """Mirror a checkpoint directory into the job store (replaces the S3 sync helper)."""
    if not store_path or not os.path.isdir(local_path):
        return
    os.makedirs(store_path, exist_ok=True)
    shutil.copytree(local_path, store_path, dirs_exist_ok=True)


def sync_store_checkpoints_to_local(local_path="/opt/ml/checkpoints", store_path=None):
    if not store_path or not os.path.isdir(store_path):
        return
    os.makedirs(local_path, exist_ok=True)
    shutil.copytree(store_path, local_path, dirs_exist_ok=True)
