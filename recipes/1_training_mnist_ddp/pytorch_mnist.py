"""Single-process MNIST baseline (/root/reference/1_training_mnist_ddp/pytorch_mnist.py).

Same CLI as the DDP script; world size / rank fixed to 1 / 0 (no process group), so its output
can be diffed against the DDP run.
"""
import os
import sys

_HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, _HERE)

for k in ("WORLD_SIZE", "OMPI_COMM_WORLD_SIZE"):
    os.environ[k] = "1"
for k in ("RANK", "LOCAL_RANK", "OMPI_COMM_WORLD_RANK", "OMPI_COMM_WORLD_LOCAL_RANK"):
    os.environ[k] = "0"

import pytorch_mnist_ddp  # noqa: E402

if __name__ == "__main__":
    pytorch_mnist_ddp.main()
