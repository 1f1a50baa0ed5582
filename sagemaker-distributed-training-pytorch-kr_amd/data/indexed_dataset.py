"""Memory-mapped indexed token dataset (Megatron ``MMapIndexedDataset`` on-disk format).

The reference reads CodeParrot tokens preprocessed into ``<prefix>.bin`` / ``<prefix>.idx``
(log "reading sizes / pointers / document index ... creating numpy buffer of mmap",
NB3:1874-1880). We read AND write the same format so existing preprocessed corpora load
unchanged:

    .idx : b"MMIDIDX\\x00\\x00" | u64 version=1 | u8 dtype code | u64 n_sequences | u64 n_docs
           | i32 sizes[n_sequences] | i64 pointers[n_sequences] (byte offsets) | i64 doc_idx[n_docs]
    .bin : the token arrays back to back

Nothing is unpickled: every array is a typed ``np.frombuffer`` view of an mmap.
"""
from __future__ import annotations

import os
import struct
from typing import Iterable, Optional

import numpy as np

_MAGIC = b"MMIDIDX\x00\x00"
_DTYPES = {1: np.uint8, 2: np.int8, 3: np.int16, 4: np.int32, 5: np.int64, 6: np.float64, 7: np.float32,
           8: np.uint16}
_CODES = {np.dtype(v): k for k, v in _DTYPES.items()}


def index_file_path(prefix: str) -> str:
    return prefix + ".idx"


def data_file_path(prefix: str) -> str:
    return prefix + ".bin"


def best_fitting_dtype(vocab_size: Optional[int] = None):
    return np.uint16 if vocab_size is not None and vocab_size < 65500 else np.int32


class MMapIndexedDataset:
    """Random access to variable-length token sequences via mmap (zero copy)."""

    def __init__(self, prefix: str, skip_warmup: bool = True):
        self.prefix = prefix
        with open(index_file_path(prefix), "rb") as f:
            magic = f.read(9)
            if magic != _MAGIC:
                raise ValueError(f"{prefix}.idx: not an MMIDIDX index file")
            (version,) = struct.unpack("<Q", f.read(8))
            if version != 1:
                raise ValueError(f"unsupported index version {version}")
            (code,) = struct.unpack("<B", f.read(1))
            self.dtype = np.dtype(_DTYPES[code])
            (self._len,) = struct.unpack("<Q", f.read(8))
            (self._doc_count,) = struct.unpack("<Q", f.read(8))
            offset = f.tell()
        self._idx_mmap = np.memmap(index_file_path(prefix), mode="r", order="C")
        buf = memoryview(self._idx_mmap)
        self.sizes = np.frombuffer(buf, dtype=np.int32, count=self._len, offset=offset)
        self.pointers = np.frombuffer(buf, dtype=np.int64, count=self._len, offset=offset + self.sizes.nbytes)
        self.doc_idx = np.frombuffer(buf, dtype=np.int64, count=self._doc_count,
                                     offset=offset + self.sizes.nbytes + self.pointers.nbytes)
        self._bin_mmap = np.memmap(data_file_path(prefix), mode="r", order="C")
        self._bin = memoryview(self._bin_mmap)
        if not skip_warmup:
            _ = np.asarray(self._bin_mmap[: min(len(self._bin_mmap), 1 << 20)]).sum()

    def __len__(self):
        return self._len

    def __getitem__(self, idx):
        if isinstance(idx, (int, np.integer)):
            return np.frombuffer(self._bin, dtype=self.dtype, count=int(self.sizes[idx]),
                                 offset=int(self.pointers[idx]))
        if isinstance(idx, slice):
            return [self[i] for i in range(*idx.indices(len(self)))]
        raise TypeError(type(idx))

    def get(self, idx: int, offset: int = 0, length: Optional[int] = None):
        """Sequence ``idx``, elements [offset, offset + length) (Megatron's ``get``)."""
        size = int(self.sizes[idx])
        if length is None:
            length = size - offset
        ptr = int(self.pointers[idx]) + offset * self.dtype.itemsize
        return np.frombuffer(self._bin, dtype=self.dtype, count=int(length), offset=ptr)

    @property
    def supports_prefetch(self):
        return False

    @staticmethod
    def exists(prefix):
        return os.path.exists(index_file_path(prefix)) and os.path.exists(data_file_path(prefix))


class MMapIndexedDatasetBuilder:
    """Writes ``.bin`` incrementally and the ``.idx`` at ``finalize``."""

    def __init__(self, out_bin: str, dtype=np.int32):
        self._f = open(out_bin, "wb")
        self.dtype = np.dtype(dtype)
        self.sizes = []
        self.doc_idx = [0]

    def add_item(self, tokens: Iterable[int]):
        arr = np.asarray(tokens, dtype=self.dtype)
        self._f.write(arr.tobytes(order="C"))
        self.sizes.append(arr.size)

    def end_document(self):
        self.doc_idx.append(len(self.sizes))

    def add_doc(self, tokens):
        self.add_item(tokens)
        self.end_document()

    def finalize(self, out_idx: str):
        self._f.close()
        sizes = np.asarray(self.sizes, dtype=np.int32)
        pointers = np.zeros(len(sizes), dtype=np.int64)
        if len(sizes) > 1:
            np.cumsum(sizes[:-1].astype(np.int64) * self.dtype.itemsize, out=pointers[1:])
        with open(out_idx, "wb") as f:
            f.write(_MAGIC)
            f.write(struct.pack("<Q", 1))
            f.write(struct.pack("<B", _CODES[self.dtype]))
            f.write(struct.pack("<Q", len(sizes)))
            f.write(struct.pack("<Q", len(self.doc_idx)))
            f.write(sizes.tobytes(order="C"))
            f.write(pointers.tobytes(order="C"))
            f.write(np.asarray(self.doc_idx, dtype=np.int64).tobytes(order="C"))


def make_dataset(prefix: str, impl: str = "mmap", skip_warmup: bool = True):
    if impl not in ("mmap", "infer", "lazy", "cached"):
        raise ValueError(f"unknown data impl {impl}")
    if not MMapIndexedDataset.exists(prefix):
        raise FileNotFoundError(f"indexed dataset {prefix}.bin/.idx not found")
    return MMapIndexedDataset(prefix, skip_warmup)


def write_synthetic_corpus(prefix: str, num_docs: int, vocab_size: int = 50257, mean_len: int = 600,
                           seed: int = 1234, eod: Optional[int] = None) -> str:
    """CodeParrot-shaped synthetic corpus: documents with geometric-ish lengths, uniform tokens,
    each ending with the EOD token (GPT-2's <|endoftext|> = 50256 by default)."""
    rng = np.random.default_rng(seed)
    eod = vocab_size - 1 if eod is None else eod
    os.makedirs(os.path.dirname(os.path.abspath(prefix)), exist_ok=True)
    b = MMapIndexedDatasetBuilder(data_file_path(prefix), dtype=best_fitting_dtype(vocab_size))
    lens = np.maximum(8, rng.exponential(mean_len, size=num_docs).astype(np.int64))
    for n in lens:
        toks = rng.integers(0, vocab_size - 1, size=int(n))
        toks[-1] = eod
        b.add_doc(toks)
    b.finalize(index_file_path(prefix))
    return prefix
