"""``smddp`` process-group backend name for unmodified SageMaker data-parallel scripts.

The reference's DDP recipes do ``import smdistributed.dataparallel.torch.torch_smddp`` and then
``dist.init_process_group(backend="smddp")`` (pytorch_mnist_ddp.py:89-90,
pytorch_oxford_ddp.py:206-211). Importing this module registers the same backend name with
``torch.distributed``; its process groups are RCCL (ProcessGroupNCCL — on ROCm that IS RCCL over
xGMI) for GPU tensors and Gloo for CPU tensors, so the rest of the script (all-reduce, DDP,
barriers) runs unchanged on MI355X. SMDDP's parameter-server all-reduce exists to use EFA across
p3/p4 nodes; inside one xGMI-connected node a ring all-reduce over the 7 links is the right
algorithm, so nothing else is emulated.
"""
from __future__ import annotations

import datetime

import torch
import torch.distributed as dist

BACKEND = "smddp"
_REGISTERED = False


def _create(store, rank, size, timeout):
    timeout = timeout if isinstance(timeout, datetime.timedelta) else datetime.timedelta(seconds=float(timeout))
    if torch.cuda.is_available():
        opts = dist.ProcessGroupNCCL.Options()
        opts._timeout = timeout
        return dist.ProcessGroupNCCL(store, rank, size, opts)
    opts = dist.ProcessGroupGloo._Options()
    opts._timeout = timeout
    opts._devices = [dist.ProcessGroupGloo.create_default_device()]
    return dist.ProcessGroupGloo(store, rank, size, opts)


def register():
    global _REGISTERED
    if _REGISTERED or BACKEND in dist.Backend.backend_list:
        _REGISTERED = True
        return
    dist.Backend.register_backend(BACKEND, _create, devices=["cuda", "cpu"])
    _REGISTERED = True


register()
