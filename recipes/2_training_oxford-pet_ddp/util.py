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
import codecs
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
    """Computes the accuracy over the k top predictions for the specified values of k"""
    with torch.no_grad():
        maxk = max(topk)
        batch_size = target.size(0)
        _, pred = output.topk(maxk, 1, True, True)
        pred = pred.t()
        correct = pred.eq(target.view(1, -1).expand_as(pred)).contiguous()
        res = []
        for k in topk:
            correct_k = correct[:k].reshape(-1).float().sum(0, keepdim=True)
            res.append(correct_k.mul_(100.0 / batch_size))
        return res


def save_model(state, is_best, args):
    logger.info("Saving the model.")
    filename = os.path.join(args.model_dir, "checkpoint.pth")
    torch.save(state, filename, _use_new_zipfile_serialization=False)
    if is_best:
        shutil.copyfile(filename, os.path.join(args.model_dir, "model_best.pth"))


class AverageMeter(object):
    """Computes and stores the average and current value"""

    def __init__(self, name, fmt=":f"):
        self.name = name
        self.fmt = fmt
        self.reset()

    def reset(self):
        self.val = 0
        self.avg = 0
        self.sum = 0
        self.count = 0

    def update(self, val, n=1):
        self.val = val
        self.sum += val * n
        self.count += n
        self.avg = self.sum / self.count

    def __str__(self):
        fmtstr = "{name} {val" + self.fmt + "} ({avg" + self.fmt + "})"
        return fmtstr.format(**self.__dict__)


class ProgressMeter(object):
    def __init__(self, num_batches, meters, prefix=""):
        self.batch_fmtstr = self._get_batch_fmtstr(num_batches)
        self.meters = meters
        self.prefix = prefix

    def display(self, batch):
        entries = [self.prefix + self.batch_fmtstr.format(batch)]
        entries += [str(meter) for meter in self.meters]
        print("\t".join(entries))

    def _get_batch_fmtstr(self, num_batches):
        num_digits = len(str(num_batches // 1))
        fmt = "{:" + str(num_digits) + "d}"
        return "[" + fmt + "/" + fmt.format(num_batches) + "]"


def adjust_learning_rate(optimizer, epoch, step, len_epoch, args):
    """Step decay (x0.1 at epoch 30, 60, 80+) with a 5-epoch linear warmup."""
    factor = epoch // 30
    if epoch >= 80:
        factor = factor + 1
    lr = args.lr * (0.1 ** factor)
    if epoch < 5:
        lr = lr * float(1 + step + epoch * len_epoch) / (5.0 * len_epoch)
    if args.rank == 0:
        print("epoch = {}, step = {}, lr = {}".format(epoch, step, lr))
    for param_group in optimizer.param_groups:
        param_group["lr"] = lr


def save_history(path, history):
    history_for_json = {k: list(map(float, v)) for k, v in history.items()}
    with codecs.open(path, "w", encoding="utf-8") as f:
        json.dump(history_for_json, f, separators=(",", ":"), sort_keys=True, indent=4)


def to_python_float(t):
    if hasattr(t, "item"):
        return t.item()
    elif hasattr(t, "index"):
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
