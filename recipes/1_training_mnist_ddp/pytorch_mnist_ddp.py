"""MNIST data-parallel training on MI355X (entry point compatible with the reference recipe).

Same CLI, log lines and SageMaker contract as /root/reference/1_training_mnist_ddp/
pytorch_mnist_ddp.py: ``--batch-size --test-batch-size --epochs --lr --gamma
--seed --log-interval --save-model --verbose --data-path --backend``; rank info from
``OMPI_COMM_WORLD_*``; data from ``SM_CHANNEL_TRAINING``; "Train Epoch: ..." / "Test set: ..."
output; ``mnist_cnn.pt``.

Differences from the reference (its bugs):
  * the per-rank batch is ``batch_size * 8 // world_size`` (clamped >= 1) — the reference's
    ``batch_size //= world_size // 8`` divides by zero for world_size < 8;
  * ``set_device`` only when a GPU is present, so the CPU / gloo configuration runs;
  * only rank 0 writes ``mnist_cnn.pt``, into ``SM_MODEL_DIR`` when set (the reference wrote the
    same CWD file from every rank);
  * ``--backend smddp`` selects RCCL + the framework's bucketed xGMI reducer.
"""
from __future__ import annotations

import argparse
import os
import sys
import time

_HERE = os.path.dirname(os.path.abspath(__file__))
for _cand in (os.path.join(_HERE, "..", ".."), os.environ.get("SMDT_ROOT", "")):
    if _cand and os.path.isdir(os.path.join(_cand, "smdt_amd")) and _cand not in sys.path:
        sys.path.insert(0, os.path.abspath(_cand))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402
import torch.nn.functional as F  # noqa: E402
import torch.optim as optim  # noqa: E402
from torch.optim.lr_scheduler import StepLR  # noqa: E402

from smdt_amd.comm import init_distributed  # noqa: E402
from smdt_amd.data.mnist import MNIST  # noqa: E402
from smdt_amd.parallel.distributed import DistributedDataParallel as DDP  # noqa: E402

try:
    from model_def import Net  # recipe-local copy (the reference imports it the same way)
except ImportError:  # pragma: no cover
    from smdt_amd.models.mnist import Net


def train(args, model, device, train_loader, optimizer, epoch):
    model.train()
    for batch_idx, (data, target) in enumerate(train_loader):
        data, target = data.to(device, non_blocking=True), target.to(device, non_blocking=True)
        optimizer.zero_grad()
        output = model(data)
        loss = F.nll_loss(output, target)
        loss.backward()
        optimizer.step()
        if batch_idx % args.log_interval == 0 and args.rank == 0:
            print("Train Epoch: {} [{}/{} ({:.0f}%)]\tLoss: {:.6f}".format(
                epoch, batch_idx * len(data) * args.world_size, len(train_loader.dataset),
                100.0 * batch_idx / len(train_loader), loss.item()), flush=True)
        if args.verbose:
            print("Batch", batch_idx, "from rank", args.rank, flush=True)


def test(model, device, test_loader):
    model.eval()
    test_loss, correct = 0.0, 0
    with torch.no_grad():
        for data, target in test_loader:
            data, target = data.to(device), target.to(device)
            output = model(data)
            test_loss += F.nll_loss(output, target, reduction="sum").item()
            pred = output.argmax(dim=1, keepdim=True)
            correct += pred.eq(target.view_as(pred)).sum().item()
    test_loss /= len(test_loader.dataset)
    print("\nTest set: Average loss: {:.4f}, Accuracy: {}/{} ({:.0f}%)\n".format(
        test_loss, correct, len(test_loader.dataset), 100.0 * correct / len(test_loader.dataset)), flush=True)
    return correct / len(test_loader.dataset)


def dist_setting(args):
    _, local, world, backend = init_distributed(args.backend)
    args.world_size = world
    args.rank = dist.get_rank() if dist.is_initialized() else 0
    args.local_rank = local
    args.backend_resolved = backend
    # Reference intent: 64 per GPU at 8 GPUs/host scaled by hosts; keep the global batch of an
    # 8-GPU job (batch_size * 8) split over the actual world size.
    args.batch_size = max(args.batch_size * 8 // max(args.world_size, 1), 1) if args.world_size > 8 else args.batch_size
    return args


def check_sagemaker(args):
    if os.environ.get("SM_MODEL_DIR") is not None:
        args.data_path = os.environ.get("SM_CHANNEL_TRAINING", args.data_path)
        args.model_dir = os.environ["SM_MODEL_DIR"]
        # reference: args.save_model = SM_MODEL_DIR (truthy) under SageMaker -> the model is saved
        if args.save_model is None:
            args.save_model = True
    else:
        args.model_dir = os.getcwd()
    args.save_model = bool(args.save_model)
    return args


def main(argv=None):
    parser = argparse.ArgumentParser(description="PyTorch MNIST Example (smdt_amd)")
    parser.add_argument("--batch-size", type=int, default=64, metavar="N")
    parser.add_argument("--test-batch-size", type=int, default=1000, metavar="N")
    parser.add_argument("--epochs", type=int, default=2, metavar="N")
    parser.add_argument("--lr", type=float, default=1.0, metavar="LR")
    parser.add_argument("--gamma", type=float, default=0.7, metavar="M")
    parser.add_argument("--seed", type=int, default=1, metavar="S")
    parser.add_argument("--log-interval", type=int, default=10, metavar="N")
    parser.add_argument("--save-model", type=lambda s: str(s).lower() not in ("false", "0", "no"), nargs="?",
                        const=True, default=None)
    parser.add_argument("--verbose", type=lambda s: str(s).lower() not in ("false", "0", "no"), nargs="?",
                        const=True, default=False)
    parser.add_argument("--data-path", type=str, default="../data")
    parser.add_argument("--backend", type=str, default="nccl")
    parser.add_argument("--num-workers", type=int, default=0)
    args = parser.parse_args(argv)
    args = check_sagemaker(args)
    args = dist_setting(args)
    if args.verbose:
        print("Hello from rank", args.rank, "of local_rank", args.local_rank, "in world size of", args.world_size,
              flush=True)
    torch.manual_seed(args.seed)
    use_cuda = torch.cuda.is_available()
    device = torch.device("cuda", torch.cuda.current_device()) if use_cuda else torch.device("cpu")

    train_dataset = MNIST(args.data_path, train=True)
    train_sampler = torch.utils.data.distributed.DistributedSampler(train_dataset, num_replicas=args.world_size,
                                                                    rank=args.rank)
    train_loader = torch.utils.data.DataLoader(train_dataset, batch_size=args.batch_size, shuffle=False,
                                               num_workers=args.num_workers, pin_memory=use_cuda,
                                               sampler=train_sampler)
    test_loader = None
    if args.rank == 0:
        test_loader = torch.utils.data.DataLoader(MNIST(args.data_path, train=False),
                                                  batch_size=args.test_batch_size, shuffle=True)

    model = DDP(Net().to(device), torch_compat=True)
    optimizer = optim.Adadelta(model.parameters(), lr=args.lr)
    scheduler = StepLR(optimizer, step_size=1, gamma=args.gamma)
    t0 = time.time()
    acc = None
    for epoch in range(1, args.epochs + 1):
        train_sampler.set_epoch(epoch)
        train(args, model, device, train_loader, optimizer, epoch)
        if args.rank == 0:
            acc = test(model, device, test_loader)
        scheduler.step()
    if args.rank == 0:
        n = len(train_dataset) * args.epochs
        print(f"[smdt] train throughput: {n / (time.time() - t0):.1f} samples/s over {args.world_size} rank(s)",
              flush=True)
    if args.save_model and args.rank == 0:
        os.makedirs(args.model_dir, exist_ok=True)
        # Same keys as the reference's torch-DDP checkpoint ("module.conv1.weight", ...).
        sd = {"module." + k: v for k, v in model.module.state_dict().items()}
        torch.save(sd, os.path.join(args.model_dir, "mnist_cnn.pt"))
    if dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()
    return acc


if __name__ == "__main__":
    main()
