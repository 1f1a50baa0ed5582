"""Oxford-IIIT Pet image classification with data parallelism on MI355X.

Entry point compatible with /root/reference/2_training_oxford-pet_ddp/pytorch_oxford_ddp.py
(SURVEY R4-R6, §3.3): same flags (``--log-interval --backend --channels-last --seed -p
--model_name --height --width --lr --num-classes --num-epochs --batch-size --test-batch-size``),
``SM_CHANNEL_TRAINING`` with ``train/`` and ``val/`` (or ``test/``) ImageFolder trees,
``SM_MODEL_DIR`` outputs (``model_history.p`` JSON, ``checkpoint.pth``, ``model_best.pth``), and
the exact ``Train_Time=... Train_Speed=... Train_Loss=... Train_Prec@1=...`` /
``Test_...`` log lines the metric regexes (NB2:425-436) scrape.

MI355X-first changes:
  * ``--dtype bf16`` (default on GPU) runs the network under bf16 autocast in channels-last
    (MIOpen NHWC implicit-GEMM convolutions on MFMA);
  * augmentation runs batched on the GPU (``smdt_amd.data.image_folder.GpuAugment``);
  * DDP is the framework's bucketed RCCL reducer (``--backend smddp`` is accepted);
  * validation is sharded over ranks and all-reduced (the reference evaluated the full val set
    on every rank); the step time is no longer divided by ``log_interval`` (reference bug,
    `pytorch_oxford_ddp.py:321`, that inflated Train_Speed 5x).
"""
import argparse
import logging
import os
import sys
import time

_HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, _HERE)
for _cand in (os.path.join(_HERE, "..", ".."), os.environ.get("SMDT_ROOT", "")):
    if _cand and os.path.isdir(os.path.join(_cand, "smdt_amd")) and _cand not in sys.path:
        sys.path.insert(0, os.path.abspath(_cand))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402
import torch.nn as nn  # noqa: E402
import torch.optim as optim  # noqa: E402

import util  # noqa: E402
from smdt_amd.comm import init_distributed  # noqa: E402
from smdt_amd.data.image_folder import AugmentPrefetcher, GpuAugment, ImageFolderDataset  # noqa: E402
from smdt_amd.optim.optimizer import MixedPrecisionAdam  # noqa: E402
from smdt_amd.train.graphs import CapturedStep  # noqa: E402
from smdt_amd.utils.miopen import seed_user_db  # noqa: E402
from smdt_amd.parallel.distributed import DistributedDataParallel as DDP  # noqa: E402

logger = logging.getLogger(__name__)
logger.setLevel(logging.DEBUG)
logger.addHandler(logging.StreamHandler(sys.stdout))


def str2bool(s):
    return str(s).lower() in ("true", "1", "yes", "t", "y")


def args_fn(argv=None):
    parser = argparse.ArgumentParser(description="PyTorch Resnet50 Example (smdt_amd)")
    parser.add_argument("--log-interval", type=int, default=5, metavar="N")
    parser.add_argument("--backend", type=str, default="nccl")
    parser.add_argument("--channels-last", type=str2bool, default=True)
    parser.add_argument("--seed", type=int, default=1, metavar="S")
    parser.add_argument("-p", "--print-freq", default=10, type=int, metavar="N")
    parser.add_argument("--model_name", type=str, default="resnet50")
    parser.add_argument("--height", type=int, default=224)
    parser.add_argument("--width", type=int, default=224)
    parser.add_argument("--lr", type=float, default=0.0001)
    parser.add_argument("--num-classes", type=int, default=10)
    parser.add_argument("--num-epochs", type=int, default=3)
    parser.add_argument("--batch-size", type=int, default=64)
    parser.add_argument("--test-batch-size", type=int, default=200, metavar="N")
    parser.add_argument("--dtype", type=str, default="auto", choices=["auto", "bf16", "fp32"])
    parser.add_argument("--num-workers", type=int, default=4)
    parser.add_argument("--pretrained", type=str2bool, default=True)
    parser.add_argument("--data-dir", type=str, default=None)
    parser.add_argument("--model-dir", type=str, default=None)
    parser.add_argument("--max-steps", type=int, default=0, help="stop each epoch after N steps (smoke tests)")
    parser.add_argument("--graph", type=str2bool, default=False,
                        help="capture the training step (forward, backward with the DDP bucket reductions, the "
                             "hand-written fused Adam) in a HIP graph and replay it (smdt_amd/train/graphs.py)")
    return parser.parse_args(argv)


def dist_setting(args):
    _, local, world, backend = init_distributed(args.backend)
    args.world_size = world
    args.rank = dist.get_rank() if dist.is_initialized() else 0
    args.local_rank = local
    return args


def check_sagemaker(args):
    if os.environ.get("SM_MODEL_DIR") is not None:
        args.data_dir = os.environ.get("SM_CHANNEL_TRAINING", args.data_dir)
        args.model_dir = os.environ["SM_MODEL_DIR"]
    args.model_dir = args.model_dir or os.getcwd()
    return args


def _split_dir(root, names):
    for n in names:
        p = os.path.join(root, n)
        if os.path.isdir(p):
            return p
    return root


def _get_train_data_loader(args):
    ds = ImageFolderDataset(_split_dir(args.data_dir, ("train",)), (args.height, args.width))
    sampler = torch.utils.data.distributed.DistributedSampler(ds, num_replicas=args.world_size, rank=args.rank)
    dl = torch.utils.data.DataLoader(ds, batch_size=args.batch_size, sampler=sampler, num_workers=args.num_workers,
                                     pin_memory=torch.cuda.is_available(), drop_last=False,
                                     persistent_workers=args.num_workers > 0)
    return dl, sampler


def _get_test_data_loader(args):
    ds = ImageFolderDataset(_split_dir(args.data_dir, ("val", "test")), (args.height, args.width))
    sampler = torch.utils.data.distributed.DistributedSampler(ds, num_replicas=args.world_size, rank=args.rank,
                                                              shuffle=False)
    return torch.utils.data.DataLoader(ds, batch_size=args.test_batch_size, sampler=sampler,
                                       num_workers=args.num_workers, pin_memory=torch.cuda.is_available())


def train(args):
    best_acc1 = -1
    model_history = util.init_modelhistory({})
    model = util.torch_model(args.model_name, num_classes=args.num_classes, pretrained=args.pretrained)
    dev = args.device
    mf = torch.channels_last if (args.channels_last and dev.type == "cuda") else torch.contiguous_format
    model = model.to(dev, memory_format=mf)
    model = DDP(model, torch_compat=True)
    criterion = nn.CrossEntropyLoss().to(dev)
    use_graph = bool(args.graph) and dev.type == "cuda"
    if use_graph:   # the same Adam (torch.optim defaults), device-side step count: capturable
        optimizer = MixedPrecisionAdam(model, lr=args.lr, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0,
                                       adamw=False, capturable=True)
    else:
        optimizer = optim.Adam(model.parameters(), lr=args.lr)
    train_loader, train_sampler = _get_train_data_loader(args)
    logger.info("Processes {}/{} ({:.0f}%) of train data".format(
        len(train_loader.sampler), len(train_loader.dataset),
        100.0 * len(train_loader.sampler) / max(len(train_loader.dataset), 1)))
    test_loader = _get_test_data_loader(args)
    logger.info("Processes {}/{} ({:.0f}%) of test data".format(
        len(test_loader.sampler), len(test_loader.dataset),
        100.0 * len(test_loader.sampler) / max(len(test_loader.dataset), 1)))
    print(" local_rank : {}, local_batch_size : {}".format(args.local_rank, args.batch_size))
    use_bf16 = args.dtype == "bf16" or (args.dtype == "auto" and dev.type == "cuda")
    aug_train = GpuAugment((args.height, args.width), train=True, channels_last=mf == torch.channels_last)
    aug_eval = GpuAugment((args.height, args.width), train=False, channels_last=mf == torch.channels_last)
    gen = torch.Generator(device=dev)
    gen.manual_seed(args.seed + args.rank)

    def train_step(data, target):
        optimizer.zero_grad()
        with torch.autocast(device_type=dev.type, dtype=torch.bfloat16, enabled=use_bf16,
                            cache_enabled=not use_graph):
            output = model(data)
            loss = criterion(output.float(), target)
        loss.backward()
        optimizer.step()
        return output, loss
    step = CapturedStep(train_step, enabled=use_graph)

    for epoch in range(1, args.num_epochs + 1):
        batch_time = util.AverageMeter("Time", ":6.3f")
        losses = util.AverageMeter("Loss", ":.4e")
        top1 = util.AverageMeter("Acc@1", ":6.2f")
        top5 = util.AverageMeter("Acc@5", ":6.2f")
        model.train()
        train_sampler.set_epoch(epoch)
        end = time.time()
        # batches are moved and augmented ahead of the step on a side stream (GpuAugment's per-sample
        # transform picks round-trip to the host; in line they stalled the step's launches)
        for batch_idx, (data, target) in enumerate(AugmentPrefetcher(train_loader, aug_train, dev, gen)):
            if args.max_steps and batch_idx >= args.max_steps:
                break
            output, loss = step(data, target)
            if args.rank == 0:
                prec1, prec5 = util.accuracy(output, target, topk=(1, min(5, args.num_classes)))
                losses.update(util.to_python_float(loss), data.size(0))
                top1.update(util.to_python_float(prec1), data.size(0))
                top5.update(util.to_python_float(prec5), data.size(0))
                if dev.type == "cuda":
                    torch.cuda.synchronize()
                batch_time.update(time.time() - end)
                end = time.time()
                if batch_idx % args.log_interval == 0:
                    print("Epoch: [{0}][{1}/{2}] "
                          "Train_Time={batch_time.val:.3f}: avg-{batch_time.avg:.3f}, "
                          "Train_Speed={3:.3f} ({4:.3f}), "
                          "Train_Loss={loss.val:.10f}:({loss.avg:.4f}), "
                          "Train_Prec@1={top1.val:.3f}:({top1.avg:.3f}), "
                          "Train_Prec@5={top5.val:.3f}:({top5.avg:.3f})".format(
                              epoch, batch_idx, len(train_loader),
                              args.world_size * args.batch_size / batch_time.val,
                              args.world_size * args.batch_size / batch_time.avg,
                              batch_time=batch_time, loss=losses, top1=top1, top5=top5), flush=True)
                model_history["epoch"].append(epoch)
                model_history["batch_idx"].append(batch_idx)
                model_history["batch_time"].append(batch_time.val)
                model_history["losses"].append(losses.val)
                model_history["top1"].append(top1.val)
                model_history["top5"].append(top5.val)
        if epoch == 1 and use_graph and args.rank == 0:
            logger.info("training step HIP graph: {}".format(step.note))
        acc1 = validate(test_loader, model, criterion, epoch, model_history, args, aug_eval, use_bf16)
        if args.rank == 0:
            is_best = acc1 > best_acc1
            best_acc1 = max(acc1, best_acc1)
            os.makedirs(args.model_dir, exist_ok=True)
            util.save_history(os.path.join(args.model_dir, "model_history.p"), model_history)
            util.save_model({
                "epoch": epoch + 1, "model_name": args.model_name,
                "state_dict": {"module." + k: v for k, v in model.module.state_dict().items()},
                "best_acc1": best_acc1, "optimizer": optimizer.state_dict(),
                "class_to_idx": train_loader.dataset.class_to_idx}, is_best, args)
        if dist.is_initialized():
            dist.barrier()
    return best_acc1


def validate(val_loader, model, criterion, epoch, model_history, args, aug, use_bf16):
    batch_time = util.AverageMeter("Time", ":6.3f")
    losses = util.AverageMeter("Loss", ":.4e")
    top1 = util.AverageMeter("Acc@1", ":6.2f")
    top5 = util.AverageMeter("Acc@5", ":6.2f")
    model.eval()
    dev = args.device
    end = time.time()
    tot = torch.zeros(4, dtype=torch.float64, device=dev)  # loss_sum, top1_sum, top5_sum, count
    for batch_idx, (data, target) in enumerate(val_loader):
        data = aug(data.to(dev))
        target = target.to(dev)
        with torch.no_grad(), torch.autocast(device_type=dev.type, dtype=torch.bfloat16, enabled=use_bf16):
            output = model(data)
            loss = criterion(output.float(), target)
        prec1, prec5 = util.accuracy(output, target, topk=(1, min(5, args.num_classes)))
        n = data.size(0)
        tot += torch.stack([loss.double() * n, prec1.double().squeeze() * n, prec5.double().squeeze() * n,
                            torch.tensor(float(n), dtype=torch.float64, device=dev)])
        losses.update(util.to_python_float(loss), n)
        top1.update(util.to_python_float(prec1), n)
        top5.update(util.to_python_float(prec5), n)
        batch_time.update(time.time() - end)
        end = time.time()
        if args.rank == 0:
            print("Test: [{0}/{1}]  "
                  "Test_Time={batch_time.val:.3f}:({batch_time.avg:.3f}), "
                  "Test_Speed={2:.3f}:({3:.3f}), "
                  "Test_Loss={loss.val:.4f}:({loss.avg:.4f}), "
                  "Test_Prec@1={top1.val:.3f}:({top1.avg:.3f}), "
                  "Test_Prec@5={top5.val:.3f}:({top5.avg:.3f})".format(
                      batch_idx, len(val_loader), args.world_size * args.test_batch_size / batch_time.val,
                      args.world_size * args.test_batch_size / batch_time.avg, batch_time=batch_time,
                      loss=losses, top1=top1, top5=top5), flush=True)
            model_history["val_epoch"].append(epoch)
            model_history["val_batch_idx"].append(batch_idx)
            model_history["val_batch_time"].append(batch_time.val)
            model_history["val_losses"].append(losses.val)
            model_history["val_top1"].append(top1.val)
            model_history["val_top5"].append(top5.val)
    if dist.is_initialized():
        dist.all_reduce(tot)
    cnt = max(tot[3].item(), 1.0)
    avg_loss, avg1, avg5 = tot[0].item() / cnt, tot[1].item() / cnt, tot[2].item() / cnt
    model_history["val_avg_epoch"].append(epoch)
    model_history["val_avg_batch_time"].append(batch_time.avg)
    model_history["val_avg_losses"].append(avg_loss)
    model_history["val_avg_top1"].append(avg1)
    model_history["val_avg_top5"].append(avg5)
    if args.rank == 0:
        print(f" * Acc@1 {avg1:.3f} Acc@5 {avg5:.3f} (all ranks)", flush=True)
    return avg1


def main(argv=None):
    print("start main function")
    # MIOpen's find / perf databases of this recipe's models on gfx950, seeded before the first
    # convolution: a fresh job skips the per-config solver search (utils/miopen.py)
    seed_user_db()
    args = args_fn(argv)
    args = check_sagemaker(args)
    args = dist_setting(args)
    args.device = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")
    torch.manual_seed(args.seed)
    acc = train(args)
    if dist.is_initialized():
        dist.destroy_process_group()
    return acc


if __name__ == "__main__":
    main()
