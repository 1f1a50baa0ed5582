"""MNIST without torchvision: IDX reader + synthetic generator.

The reference loads ``torchvision.datasets.MNIST(data_path, train, download=False)`` from the
``training`` channel (/root/reference/1_training_mnist_ddp/pytorch_mnist_ddp.py:216-255) with
``Normalize((0.1307,), (0.3081,))``. torchvision is not part of this stack, so ``MNIST`` reads
the same on-disk files (``<root>/MNIST/raw/{train,t10k}-{images-idx3,labels-idx1}-ubyte[.gz]``
or the same names directly under ``<root>``) into uint8 tensors once and normalises on the fly.
``write_synthetic_mnist`` produces a learnable IDX dataset (class-dependent stroke patterns) for
offline tests.
"""
from __future__ import annotations

import gzip
import os
import struct

import numpy as np
import torch

MEAN, STD = 0.1307, 0.3081
_FILES = {True: ("train-images-idx3-ubyte", "train-labels-idx1-ubyte"),
          False: ("t10k-images-idx3-ubyte", "t10k-labels-idx1-ubyte")}


def _open(path):
    if os.path.exists(path):
        return open(path, "rb")
    if os.path.exists(path + ".gz"):
        return gzip.open(path + ".gz", "rb")
    raise FileNotFoundError(path)


def _find(root, name):
    for d in (os.path.join(root, "MNIST", "raw"), os.path.join(root, "raw"), root):
        if os.path.exists(os.path.join(d, name)) or os.path.exists(os.path.join(d, name + ".gz")):
            return os.path.join(d, name)
    raise FileNotFoundError(f"{name} not found under {root}")


def read_idx(path) -> np.ndarray:
    with _open(path) as f:
        data = f.read()
    magic = struct.unpack(">I", data[:4])[0]
    ndim = magic & 0xFF
    dims = struct.unpack(">" + "I" * ndim, data[4:4 + 4 * ndim])
    arr = np.frombuffer(data, dtype=np.uint8, offset=4 + 4 * ndim)
    return arr.reshape(dims)


def write_idx(path, arr: np.ndarray):
    arr = np.ascontiguousarray(arr, dtype=np.uint8)
    with open(path, "wb") as f:
        f.write(struct.pack(">I", 0x0800 | arr.ndim))
        f.write(struct.pack(">" + "I" * arr.ndim, *arr.shape))
        f.write(arr.tobytes())


class MNIST(torch.utils.data.Dataset):
    def __init__(self, root, train=True, normalize=True):
        img_name, lbl_name = _FILES[bool(train)]
        self.images = torch.from_numpy(read_idx(_find(root, img_name)).copy())
        self.targets = torch.from_numpy(read_idx(_find(root, lbl_name)).astype(np.int64))
        assert self.images.shape[0] == self.targets.shape[0]
        self.normalize = normalize

    def __len__(self):
        return self.images.shape[0]

    def __getitem__(self, i):
        x = self.images[i].float().div_(255.0).unsqueeze(0)
        if self.normalize:
            x = (x - MEAN) / STD
        return x, int(self.targets[i])


def write_synthetic_mnist(root, n_train=6000, n_test=1000, seed=0):
    """Class-conditional 28x28 digits-like patterns (bars at class-specific positions + noise)."""
    rng = np.random.default_rng(seed)
    raw = os.path.join(root, "MNIST", "raw")
    os.makedirs(raw, exist_ok=True)

    def make(n):
        y = rng.integers(0, 10, size=n)
        x = rng.integers(0, 40, size=(n, 28, 28)).astype(np.float32)
        for i, c in enumerate(y):
            r0 = 2 + 2 * c
            x[i, r0:r0 + 3, 4:24] += 200
            x[i, 4:24, 25 - 2 * c:28 - 2 * c] += 120
        return np.clip(x, 0, 255).astype(np.uint8), y.astype(np.uint8)

    xi, yi = make(n_train)
    write_idx(os.path.join(raw, "train-images-idx3-ubyte"), xi)
    write_idx(os.path.join(raw, "train-labels-idx1-ubyte"), yi)
    xt, yt = make(n_test)
    write_idx(os.path.join(raw, "t10k-images-idx3-ubyte"), xt)
    write_idx(os.path.join(raw, "t10k-labels-idx1-ubyte"), yt)
    return root
