"""GPT pretraining dataset: document split, index mappings with on-disk cache, blending.

Behaviour parity with the reference's revised Megatron dataset
(/root/reference/3_training_megatron-lm/megatron/data/gpt_dataset.py):
  * documents are split train/valid/test by the ``--split`` string ("969, 30, 1", NB3:1166);
  * each split packs documents into (seq_length + 1)-token samples: ``doc_idx`` (shuffled
    documents x epochs, last epoch kept separate when it is < 80 % used), ``sample_idx``
    (C++ ``build_sample_idx``, :433-437) and ``shuffle_idx``, cached as
    ``index-cache/<md5(desc)>_{doc,sample,shuffle}_idx.npy`` next to the data;
  * the cache is built by every node's LOCAL_RANK 0 (the reference's local revision, :371-372),
    and success is confirmed by an all-reduce over the DP and PP groups (:462-469);
  * blending of several prefixes with weights (``BlendableDataset``) uses the C++ greedy
    schedule.

Cache files are written and read with ``allow_pickle=False`` (plain typed arrays only).
"""
from __future__ import annotations

import hashlib
import math
import os
import time
from typing import List, Optional, Sequence

import numpy as np
import torch
import torch.distributed as dist

from .indexed_dataset import make_dataset
from ..parallel import state as ps


def _log(msg):
    if (not dist.is_initialized()) or dist.get_rank() == 0:
        print(msg, flush=True)


def _runtime():
    try:
        from .. import _runtime  # type: ignore
        return _runtime
    except ImportError:
        return None


# ----------------------------------------------------------------------------- split helpers

def get_train_valid_test_split_(splits_string: str, size: int) -> List[int]:
    """'969, 30, 1' -> document boundaries [0, a, b, size] proportional to the weights."""
    if "," in splits_string:
        parts = [float(s) for s in splits_string.split(",")]
    elif "/" in splits_string:
        parts = [float(s) for s in splits_string.split("/")]
    else:
        parts = [float(splits_string)]
    parts = (parts + [0.0, 0.0, 0.0])[:3]
    tot = sum(parts)
    assert tot > 0.0
    parts = [p / tot for p in parts]
    idx = [0]
    for p in parts:
        idx.append(idx[-1] + int(round(p * float(size))))
    diff = idx[-1] - size
    for i in range(1, len(idx)):
        idx[i] -= diff
    assert len(idx) == 4 and idx[-1] == size
    return idx


def get_datasets_weights_and_num_samples(data_prefix: Sequence, train_valid_test_num_samples):
    """['0.3', 'a', '0.7', 'b'] -> prefixes, normalised weights, per-dataset sample targets
    (with the 0.5 % over-sampling margin Megatron applies)."""
    assert len(data_prefix) % 2 == 0
    n = len(data_prefix) // 2
    weights = [float(data_prefix[2 * i]) for i in range(n)]
    prefixes = [str(data_prefix[2 * i + 1]).strip() for i in range(n)]
    tot = sum(weights)
    weights = [w / tot for w in weights]
    out = []
    for w in weights:
        out.append([int(math.ceil(v * w * 1.005)) for v in train_valid_test_num_samples])
    return prefixes, weights, out


# ----------------------------------------------------------------------------- index builders

def num_epochs_needed(tokens_per_epoch: int, seq_length: int, num_samples: int) -> int:
    epochs, total = 0, 0
    while True:
        epochs += 1
        total += tokens_per_epoch
        if (total - 1) // seq_length >= num_samples:
            return epochs


def build_doc_idx(documents: np.ndarray, num_epochs: int, rng: np.random.RandomState, separate_last: bool):
    if not separate_last or num_epochs == 1:
        d = np.tile(documents.astype(np.int32), num_epochs)
        rng.shuffle(d)
        return d
    first = build_doc_idx(documents, num_epochs - 1, rng, False)
    last = build_doc_idx(documents, 1, rng, False)
    return np.concatenate([first, last])


def build_sample_idx_py(sizes, doc_idx, seq_length, num_epochs, tokens_per_epoch):
    """Python twin of the C++ builder (used when the native runtime is unavailable)."""
    n = (num_epochs * tokens_per_epoch - 1) // seq_length
    out = np.zeros((n + 1, 2), dtype=np.int64)
    di, off = 0, 0
    for s in range(1, n + 1):
        rem = seq_length + 1
        while rem != 0:
            dl = int(sizes[doc_idx[di]]) - off
            rem -= dl
            if rem <= 0:
                off += rem + dl - 1
                rem = 0
            else:
                di += 1
                off = 0
        out[s] = (di, off)
    return out.astype(np.int32) if out.max(initial=0) < 2 ** 31 else out


def build_sample_idx(sizes, doc_idx, seq_length, num_epochs, tokens_per_epoch):
    rt = _runtime()
    if rt is not None:
        return rt.build_sample_idx(np.ascontiguousarray(sizes, dtype=np.int32),
                                   np.ascontiguousarray(doc_idx, dtype=np.int32), int(seq_length),
                                   int(num_epochs), int(tokens_per_epoch))
    return build_sample_idx_py(sizes, doc_idx, seq_length, num_epochs, tokens_per_epoch)


def build_shuffle_idx(num_samples: int, total_size: int, rng: np.random.RandomState):
    dt = np.uint32 if total_size < np.iinfo(np.uint32).max - 1 else np.int64
    first = np.arange(num_samples, dtype=dt)
    rng.shuffle(first)
    if num_samples == total_size:
        return first
    last = np.arange(num_samples, total_size, dtype=dt)
    rng.shuffle(last)
    return np.concatenate([first, last])


def _index_mappings(name, data_prefix, documents, sizes, splits_string, num_samples, seq_length, seed,
                    data_cache_path=None):
    tokens_per_epoch = int(np.sum(sizes[documents]))
    epochs = num_epochs_needed(tokens_per_epoch, seq_length, num_samples)
    rng = np.random.RandomState(seed=seed)
    desc = (f"GPT Dataset\n\nData prefix {data_prefix}\nDataset name {name}\nNumber of samples {num_samples}\n"
            f"Sequence length {seq_length}\nRandom seed {seed}\nSplit {splits_string}\n")
    h = hashlib.md5(desc.encode("utf-8")).hexdigest()
    dirs = [os.path.join(os.path.dirname(data_prefix), "index-cache")]
    if data_cache_path:
        dirs.append(data_cache_path)
    paths = None
    for d in dirs:
        cand = {k: os.path.join(d, f"{h}{suf}") for k, suf in
                (("desc", ".dsc"), ("doc", "_doc_idx.npy"), ("sample", "_sample_idx.npy"), ("shuffle", "_shuffle_idx.npy"))}
        paths = cand
        if all(os.path.isfile(p) for p in cand.values()):
            break
    build = not all(os.path.isfile(p) for p in paths.values())
    ok = 1
    local_rank = int(os.environ.get("LOCAL_RANK", os.environ.get("OMPI_COMM_WORLD_LOCAL_RANK", "0")))
    if build and local_rank == 0:
        _log(" > building GPT index mappings (doc/sample/shuffle) ...")
        try:
            if epochs == 1:
                separate = False
            else:
                n_minus1 = ((epochs - 1) * tokens_per_epoch - 1) // seq_length
                last_n = num_samples - n_minus1
                per_epoch = (tokens_per_epoch - 1) // seq_length
                assert 0 <= last_n <= per_epoch + 1
                separate = last_n < int(0.80 * per_epoch)
            os.makedirs(os.path.dirname(paths["desc"]), exist_ok=True)
            t = time.time()
            doc_idx = build_doc_idx(documents, epochs, rng, separate)
            sample_idx = build_sample_idx(sizes, doc_idx, seq_length, epochs, tokens_per_epoch)
            n_shuffle = (((epochs - 1) * tokens_per_epoch - 1) // seq_length) if separate else sample_idx.shape[0] - 1
            shuffle_idx = build_shuffle_idx(n_shuffle, sample_idx.shape[0] - 1, rng)
            tmp = {k: p + f".tmp{os.getpid()}" for k, p in paths.items()}
            with open(tmp["desc"], "wt") as f:
                f.write(desc)
            for key, arr in (("doc", doc_idx), ("sample", sample_idx), ("shuffle", shuffle_idx)):
                with open(tmp[key], "wb") as f:
                    np.save(f, arr, allow_pickle=False)
            for k in paths:  # atomic publish: other nodes never see half-written files
                os.replace(tmp[k], paths[k])
            _log(f" > built {sample_idx.shape[0] - 1} samples in {time.time() - t:.3f} s")
        except OSError as e:
            _log(f" > could not write index cache {os.path.dirname(paths['desc'])}: {e}")
            ok = 0
    if dist.is_initialized():
        st = ps.get_state()
        dev = torch.device("cuda", torch.cuda.current_device()) if (torch.cuda.is_available() and dist.get_backend() in ("nccl", "smddp")) else torch.device("cpu")
        c = torch.tensor([ok], dtype=torch.long, device=dev)
        dist.barrier()
        dist.all_reduce(c)  # world: every rank must see the files (node-local builders)
        if c.item() != dist.get_world_size():
            raise RuntimeError("data index creation unsuccessful on some rank")
    doc_idx = np.load(paths["doc"], allow_pickle=False, mmap_mode="r")
    sample_idx = np.load(paths["sample"], allow_pickle=False, mmap_mode="r")
    shuffle_idx = np.load(paths["shuffle"], allow_pickle=False, mmap_mode="r")
    return doc_idx, sample_idx, shuffle_idx, desc, h, epochs


class GPTDataset(torch.utils.data.Dataset):
    def __init__(self, name, data_prefix, documents, indexed_dataset, splits_string, num_samples, seq_length,
                 seed, return_doc_ids=False, data_cache_path=None):
        self.name = name
        self.indexed_dataset = indexed_dataset
        self.return_doc_ids = return_doc_ids
        assert documents.min() >= 0 and documents.max() < indexed_dataset.sizes.shape[0]
        (self.doc_idx, self.sample_idx, self.shuffle_idx, self.desc, self.desc_hash,
         self.num_epochs) = _index_mappings(name, data_prefix, documents, indexed_dataset.sizes, splits_string,
                                            num_samples, seq_length, seed, data_cache_path)

    def __len__(self):
        return self.sample_idx.shape[0] - 1

    def __getitem__(self, idx):
        idx = int(self.shuffle_idx[idx])
        df, dl = int(self.sample_idx[idx][0]), int(self.sample_idx[idx + 1][0])
        of, ol = int(self.sample_idx[idx][1]), int(self.sample_idx[idx + 1][1])
        ids = []
        if df == dl:
            ids.append(int(self.doc_idx[df]))
            sample = self.indexed_dataset.get(self.doc_idx[df], offset=of, length=ol - of + 1)
        else:
            ids.append(int(self.doc_idx[df]))
            parts = [self.indexed_dataset.get(self.doc_idx[df], offset=of)]
            for i in range(df + 1, dl):
                ids.append(int(self.doc_idx[i]))
                parts.append(self.indexed_dataset.get(self.doc_idx[i]))
            ids.append(int(self.doc_idx[dl]))
            parts.append(self.indexed_dataset.get(self.doc_idx[dl], length=ol + 1))
            sample = np.concatenate(parts)
        out = {"text": np.asarray(sample, dtype=np.int64)}
        if self.return_doc_ids:
            out["doc_ids"] = np.asarray(ids, dtype=np.int64)
        return out


class BlendableDataset(torch.utils.data.Dataset):
    def __init__(self, datasets, weights, size, data_cache_path=None):
        self.datasets = datasets
        self.size = int(size)
        w = np.asarray(weights, dtype=np.float64)
        w = w / w.sum()
        rt = _runtime()
        if rt is not None:
            self.dataset_index, self.dataset_sample_index = rt.build_blending_indices(w, self.size)
        else:
            di = np.zeros(self.size, dtype=np.uint8)
            dsi = np.zeros(self.size, dtype=np.int64)
            cur = np.zeros(len(w), dtype=np.int64)
            for i in range(self.size):
                err = w * (i + 1) - cur
                k = int(np.argmax(err))
                di[i], dsi[i] = k, cur[k]
                cur[k] += 1
            self.dataset_index, self.dataset_sample_index = di, dsi

    def __len__(self):
        return self.size

    def __getitem__(self, idx):
        d = int(self.dataset_index[idx])
        s = int(self.dataset_sample_index[idx])
        return self.datasets[d][s % len(self.datasets[d])]


def _split_datasets(prefix, data_impl, splits_string, num_samples3, seq_length, seed, skip_warmup, cache):
    ds = make_dataset(prefix, data_impl, skip_warmup)
    total = ds.sizes.shape[0]
    b = get_train_valid_test_split_(splits_string, total)
    _log(f" > dataset split of {prefix}: train [{b[0]}, {b[1]}) valid [{b[1]}, {b[2]}) test [{b[2]}, {b[3]})")
    out = []
    for i, name in enumerate(("train", "valid", "test")):
        if b[i + 1] > b[i] and num_samples3[i] > 0:
            docs = np.arange(b[i], b[i + 1], dtype=np.int32)
            out.append(GPTDataset(name, prefix, docs, ds, splits_string, num_samples3[i], seq_length, seed,
                                  data_cache_path=cache))
        else:
            out.append(None)
    return tuple(out)


def build_train_valid_test_datasets(data_prefix, data_impl, splits_string, train_valid_test_num_samples, seq_length,
                                    seed, skip_warmup=True, train_data_prefix=None, valid_data_prefix=None,
                                    test_data_prefix=None, data_cache_path=None):
    """Megatron's entry point (called by ``pretrain_gpt.train_valid_test_datasets_provider``)."""
    if data_prefix:
        if len(data_prefix) == 1:
            return _split_datasets(data_prefix[0], data_impl, splits_string, train_valid_test_num_samples,
                                   seq_length, seed, skip_warmup, data_cache_path)
        prefixes, weights, per = get_datasets_weights_and_num_samples(data_prefix, train_valid_test_num_samples)
        parts = [_split_datasets(p, data_impl, splits_string, per[i], seq_length, seed, skip_warmup, data_cache_path)
                 for i, p in enumerate(prefixes)]
        out = []
        for j in range(3):
            dsets = [p[j] for p in parts if p[j] is not None]
            out.append(BlendableDataset(dsets, weights[:len(dsets)], train_valid_test_num_samples[j]) if dsets else None)
        return tuple(out)

    def single(prefix, n, name):
        if prefix is None or n <= 0:
            return None
        p = prefix[0] if isinstance(prefix, (list, tuple)) else prefix
        ds = make_dataset(p, data_impl, skip_warmup)
        docs = np.arange(ds.sizes.shape[0], dtype=np.int32)
        return GPTDataset(name, p, docs, ds, splits_string, n, seq_length, seed, data_cache_path=data_cache_path)

    n3 = train_valid_test_num_samples
    return (single(train_data_prefix, n3[0], "train"), single(valid_data_prefix, n3[1], "valid"),
            single(test_data_prefix, n3[2], "test"))


class SyntheticGPTDataset(torch.utils.data.Dataset):
    """Deterministic random tokens of shape [seq_length + 1] (benchmarks, smoke tests)."""

    def __init__(self, num_samples, seq_length, vocab_size, seed=1234):
        self.n, self.s, self.v, self.seed = int(num_samples), int(seq_length), int(vocab_size), seed

    def __len__(self):
        return self.n

    def __getitem__(self, idx):
        rng = np.random.default_rng(self.seed + int(idx))
        return {"text": rng.integers(0, self.v, size=self.s + 1, dtype=np.int64)}


# ----------------------------------------------------------------------------- samplers

class MegatronPretrainingSampler:
    """Sequential, resumable (``consumed_samples``) micro-batch index sampler sharded over DP."""

    def __init__(self, total_samples, consumed_samples, micro_batch_size, data_parallel_rank, data_parallel_size,
                 drop_last=True):
        self.total, self.consumed = total_samples, consumed_samples
        self.mbs, self.rank, self.size = micro_batch_size, data_parallel_rank, data_parallel_size
        self.drop_last = drop_last
        assert self.total > 0 and self.consumed < self.total and self.rank < self.size

    def __len__(self):
        return self.total

    def __iter__(self):
        batch = []
        gb = self.mbs * self.size
        for idx in range(self.consumed, self.total):
            batch.append(idx)
            if len(batch) == gb:
                yield batch[self.rank * self.mbs:(self.rank + 1) * self.mbs]
                batch = []
        if batch and not self.drop_last:
            s = self.rank * self.mbs
            yield batch[s:s + self.mbs]


def build_pretraining_data_loader(dataset, consumed_samples, micro_batch_size, num_workers=2):
    if dataset is None:
        return None
    st = ps.get_state()
    sampler = MegatronPretrainingSampler(len(dataset), consumed_samples, micro_batch_size, st.dp_rank, st.dp)
    return torch.utils.data.DataLoader(dataset, batch_sampler=sampler, num_workers=num_workers, pin_memory=True,
                                       persistent_workers=num_workers > 0)
