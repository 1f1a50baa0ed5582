"""Oxford-Pet DDP training throughput (BASELINE config #2 / NB2) on synthetic images.

One training step is exactly the recipe's (`recipes/2_training_oxford-pet_ddp/pytorch_oxford_ddp.py`
train loop, reference `2_training_oxford-pet_ddp/pytorch_oxford_ddp.py:268-330`): uint8 batch on the
GPU -> batched GPU augmentation -> bf16 autocast channels-last forward -> fp32 CE -> backward with
the framework's bucketed DDP reducer -> torch Adam (fused). Images are random uint8 of the
reference's shape; weights are random init (no network for datasets / checkpoints).

    python benchmarks/bench_vision.py --model swin_b --size 128 --batch 40      # NB2 per-GPU config
    python benchmarks/bench_vision.py --model resnet50 --size 224 --batch 64    # recipe default
    torchrun --nproc-per-node N --master-addr 127.0.0.1 benchmarks/bench_vision.py ...

Prints one JSON line (rank 0): whole-job images/s, timed over --steps after --warmup, max over
ranks. The reference published ~1,429 img/s for swin_b fp32 128x128 on 16x V100 (BASELINE.md,
NB2:3333 corrected for its log_interval division).
"""
import argparse
import itertools
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402
import torch.nn as nn  # noqa: E402

from smdt_amd.comm import init_distributed  # noqa: E402
from smdt_amd.data.image_folder import AugmentPrefetcher, GpuAugment  # noqa: E402
from smdt_amd.models import zoo  # noqa: E402
from smdt_amd.parallel.distributed import DistributedDataParallel as DDP  # noqa: E402

REF_IMG_S_PER_GPU = {"swin_b": 1429.0 / 16}  # NB2, 16x V100, fp32


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--model", default="swin_b")
    p.add_argument("--size", type=int, default=128)
    p.add_argument("--batch", type=int, default=40, help="per-GPU batch")
    p.add_argument("--num-classes", type=int, default=37)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    p.add_argument("--channels-last", type=int, default=1)
    p.add_argument("--ddp", default="smdt", choices=["smdt", "none"],
                   help="none: the bare module (MIOpen solver diagnosis at one GPU)")
    p.add_argument("--bucket-mb", type=float, default=0.0,
                   help="DDP gradient bucket size in MB of fp32 gradients (0: auto, comm/buckets.py)")
    p.add_argument("--prefetch", type=int, default=1,
                   help="augment the next batches on a side stream in a background thread "
                        "(data/image_folder.AugmentPrefetcher); 0: in line with the step")
    p.add_argument("--graph", type=int, default=1,
                   help="(default on, any world size) capture forward + backward (DDP bucket reductions "
                        "included: RCCL / loopback collectives are captured, the xGMI engine sits out "
                        "the capture) + Adam of one step in a HIP graph after the warm-up and replay it "
                        "(the step's ~1.5-3.7 k kernel launches leave the device idle 5-42 ms per step "
                        "in eager mode, profiles/r4_vision/); the augmented batch is copied into the "
                        "graph's static input")
    p.add_argument("--optim", default="smdt", choices=["smdt", "torch"],
                   help="smdt: the hand-written fused Adam (optim.hip, device-side step count: "
                        "capturable) over the DDP's flat buffers; torch: torch.optim.Adam(fused)")
    p.add_argument("--emulate-dp", type=int, default=0,
                   help="one process = rank 0 of an N-GPU DDP job (loopback DP group, comm/loopback.py): "
                        "the rank's exact per-step work with the collectives as local stand-ins; the JSON "
                        "line then reports the rank's ms/step, not a job throughput")
    p.add_argument("--miopen-prewarm", type=int, default=0,
                   help="before timing, run 13 steps in a child process so MIOpen's find database and "
                        "kernel cache exist. Round 4 needed it (a first process ran 418-540 ms per "
                        "ResNet-50 step for its whole life, profiles/r4_vision/; the MIOpen grouped-conv "
                        "augmentation behind that is gone); since round 5 a fresh process runs at the "
                        "warm rate and the shipped find / perf db (utils/miopen.py) cuts its start-up "
                        "84 -> 22 s (profiles/r5_miopen/), so it is off by default")
    a = p.parse_args()
    from smdt_amd.utils.miopen import seed_user_db
    seed_user_db()
    # (device_count() does not initialise the GPU in this process)
    if (a.miopen_prewarm and torch.cuda.device_count() > 0 and os.environ.get("LOCAL_RANK", "0") == "0"
            and not os.environ.get("SMDT_VISION_PREWARM")):
        # a child process, started before this one touches the GPU
        cmd = [sys.executable, os.path.abspath(__file__), "--model", a.model, "--size", str(a.size),
               "--batch", str(a.batch), "--steps", "10", "--warmup", "3", "--dtype", a.dtype,
               "--channels-last", str(a.channels_last), "--ddp", "none", "--prefetch", "0", "--miopen-prewarm", "0"]
        env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE",
                                                                 "MASTER_ADDR", "MASTER_PORT")}
        env["SMDT_VISION_PREWARM"] = "1"
        t = time.perf_counter()
        r = subprocess.run(cmd, env=env, capture_output=True, text=True)
        print(f"[bench_vision] MIOpen prewarm process: rc {r.returncode}, {time.perf_counter() - t:.1f}s",
              file=sys.stderr, flush=True)
    if a.emulate_dp > 1:
        from smdt_amd.parallel import state as ps
        if torch.cuda.is_available():
            torch.cuda.set_device(0)
        ps.initialize_emulated_tensor_parallel(1, a.emulate_dp)
        rank, world = 0, 1
    else:
        rank, local, world, _ = init_distributed("nccl")
    dev = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")
    torch.manual_seed(0)
    torch.backends.cudnn.benchmark = True
    model = zoo.create(a.model)
    zoo.reset_classifier(model, a.num_classes)
    mf = torch.channels_last if (a.channels_last and dev.type == "cuda") else torch.contiguous_format
    bucket = int(a.bucket_mb * 2 ** 20 / 4) if a.bucket_mb > 0 else "auto"
    model = model.to(dev, memory_format=mf)
    if a.ddp == "smdt":
        model = DDP(model, torch_compat=True, bucket_size=bucket)
    crit = nn.CrossEntropyLoss()
    use_graph = bool(a.graph) and dev.type == "cuda"
    if a.optim == "smdt" and a.ddp == "smdt":
        from smdt_amd.optim.optimizer import MixedPrecisionAdam
        # torch.optim.Adam's defaults (L2 weight decay 0), the reference's optimizer (pytorch_oxford_ddp.py:258)
        opt = MixedPrecisionAdam(model, lr=1e-4, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, adamw=False,
                                 capturable=use_graph)
    else:
        opt = torch.optim.Adam(model.parameters(), lr=1e-4, fused=dev.type == "cuda", capturable=use_graph)
    aug = GpuAugment((a.size, a.size), train=True, channels_last=mf == torch.channels_last)
    gen = torch.Generator(device=dev)
    gen.manual_seed(rank)
    # uint8 source images slightly larger than the crop (decoding is the dataloader's job)
    src = torch.randint(0, 256, (a.batch, 3, a.size + a.size // 4, a.size + a.size // 4), dtype=torch.uint8,
                        device=dev)
    tgt = torch.randint(0, a.num_classes, (a.batch,), device=dev)
    bf16 = a.dtype == "bf16"

    batches = iter(AugmentPrefetcher(itertools.repeat((src, tgt)), aug, dev, gen)) if a.prefetch else None

    def train(x):
        with torch.autocast(device_type=dev.type, dtype=torch.bfloat16, enabled=bf16, cache_enabled=not use_graph):
            out = model(x)
            loss = crit(out.float(), tgt)
        loss.backward()
        opt.step()
        return loss

    def step():
        x = next(batches)[0] if batches is not None else aug(src, gen)
        opt.zero_grad(set_to_none=True)
        return train(x)

    graph = None

    def capture():
        # whole-step capture: warm-up replays on a side stream, then one captured step; the
        # gradients live in the graph's pool and every replay rewrites them
        nonlocal graph
        static_x = next(batches)[0].clone() if batches is not None else aug(src, gen)
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(3):
                opt.zero_grad(set_to_none=True)
                train(static_x)
        torch.cuda.current_stream().wait_stream(side)
        g = torch.cuda.CUDAGraph()
        opt.zero_grad(set_to_none=True)
        with torch.cuda.graph(g):
            static_loss = train(static_x)
        graph = (g, static_x, static_loss)

    def graph_step():
        g, static_x, static_loss = graph
        x = next(batches)[0] if batches is not None else aug(src, gen)
        static_x.copy_(x)
        g.replay()
        return static_loss

    tw = time.perf_counter()
    for i in range(a.warmup):
        step()
        if rank == 0:
            print(f"[bench_vision] warmup {i + 1}/{a.warmup} at {time.perf_counter() - tw:.1f}s", file=sys.stderr,
                  flush=True)
    graph_note = None
    if use_graph:
        try:
            capture()
            for _ in range(2):
                graph_step()
            graph_note = "captured"
        except Exception as e:  # noqa: BLE001 - report and run eager
            graph_note = f"capture failed, eager: {type(e).__name__}: {str(e)[:120]}"
            print(f"[bench_vision] {graph_note}", file=sys.stderr, flush=True)
            graph = None
            torch.cuda.synchronize()
    run = graph_step if graph is not None else step
    if dist.is_initialized():
        dist.barrier()
    if dev.type == "cuda":
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        loss = run()
    if dev.type == "cuda":
        torch.cuda.synchronize()
    if dist.is_initialized():
        dist.barrier()
    el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
    if dist.is_initialized():
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    el = float(el.item())
    ips = a.batch * world * a.steps / el
    if rank == 0:
        ref = REF_IMG_S_PER_GPU.get(a.model)
        ms = round(1000 * el / a.steps, 3)
        if a.emulate_dp > 1:   # one rank of a larger job: its time, never a job throughput
            head = {"metric": "emulated rank ms/step", "value": ms, "unit": "ms", "n_gpus": 1,
                    "emulated_dp": a.emulate_dp, "rank_images_per_s": round(ips, 1)}
        else:
            head = {"metric": "Oxford-Pet DDP train images/sec (whole job)", "value": round(ips, 1),
                    "unit": "images/s", "n_gpus": world}
        print(json.dumps({
            **head, "steps": a.steps, "warmup": a.warmup, "ms_per_step": ms,
            "dtype": a.dtype, "data": "synthetic uint8 images + GPU augmentation; random-init weights",
            "config": {"model": a.model, "image": a.size, "batch_per_gpu": a.batch,
                       "channels_last": bool(a.channels_last),
                       "parallelism": f"dp{a.emulate_dp} (one emulated rank)" if a.emulate_dp > 1 else f"dp{world}",
                       "optimizer": "smdt fused Adam (optim.hip)" if a.optim == "smdt" and a.ddp == "smdt" else "torch Adam (fused)",
                       "augment": "prefetched (side stream)" if a.prefetch else "in line",
                       "hip_graph": graph_note,
                       "backend": dist.get_backend() if dist.is_initialized() else None,
                       "ddp_bucket": {"elements": model.bucket_size, "count": len(model.buckets),
                                      "MB": round(model.bucket_size * 4 / 2 ** 20, 2)} if a.ddp == "smdt" else None},
            "vs_reference_per_gpu": round(ips / world / ref, 2) if (ref and a.emulate_dp <= 1) else None,
            "final_loss": float(loss.item())}), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
