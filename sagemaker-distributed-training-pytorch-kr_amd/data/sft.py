"""Supervised fine-tuning data (Alpaca instruction format) — SURVEY R11.

Behaviour follows /root/reference/4_training_alpaca_deepspeed/train.py:
  * prompt templates with / without ``input`` (train.py:53-64), target = output + EOS (:168);
  * tokenisation truncated to ``model_max_length`` and prompt tokens masked to ``IGNORE_INDEX``
    in the labels (:115-151);
  * the collator right-pads ``input_ids`` with the pad id and ``labels`` with -100 and builds
    ``attention_mask = input_ids != pad`` (:183-199).

MI355X-specific differences (semantics-preserving):
  * the collator can pad the batch length up to a multiple (128 by default) so every micro-batch
    takes the flash-attention kernel (S % 128 == 0); with right padding + causal masking the extra
    pad tokens are never attended by a real token and carry label -100, so the loss is identical;
  * tokenisation is done once (by local rank 0 when a cache dir is given) into int32 arrays and
    shared through an ``.npz`` cache instead of every rank re-tokenising 52K examples
    (the reference re-tokenises on all 16 ranks, NB4:1613);
  * ``LengthGroupedSampler`` (HF ``--group_by_length``) batches similar lengths together.

Offline: when no HF tokenizer files are available locally, ``load_tokenizer`` returns
``HashWordTokenizer`` — a deterministic word-piece stand-in with the real vocab size and special
ids, so shapes/lengths (≈ 1 token per word or punctuation mark) stay representative.
"""
from __future__ import annotations

import hashlib
import io
import json
import logging
import os
import random
import re
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch
from torch.utils.data import Dataset, Sampler

IGNORE_INDEX = -100
DEFAULT_PAD_TOKEN = "[PAD]"
DEFAULT_EOS_TOKEN = "</s>"
DEFAULT_BOS_TOKEN = "<s>"
DEFAULT_UNK_TOKEN = "<unk>"

PROMPT_DICT = {
    "prompt_input": (
        "Below is an instruction that describes a task, paired with an input that provides further context. "
        "Write a response that appropriately completes the request.\n\n"
        "### Instruction:\n{instruction}\n\n### Input:\n{input}\n\n### Response:"
    ),
    "prompt_no_input": (
        "Below is an instruction that describes a task. "
        "Write a response that appropriately completes the request.\n\n"
        "### Instruction:\n{instruction}\n\n### Response:"
    ),
}

log = logging.getLogger("smdt.sft")


# ------------------------------------------------------------------------------- json helpers
def _make_r_io_base(f, mode: str):
    if not isinstance(f, io.IOBase):
        f = open(f, mode=mode)
    return f


def jload(f, mode="r"):
    """Load a .json file (list of dicts) — stanford_alpaca ``utils.jload``."""
    f = _make_r_io_base(f, mode)
    d = json.load(f)
    f.close()
    return d


def jdump(obj, f, mode="w", indent=4, default=str):
    if not isinstance(f, io.IOBase):
        d = os.path.dirname(f)
        if d:
            os.makedirs(d, exist_ok=True)
        f = open(f, mode=mode)
    if isinstance(obj, (dict, list)):
        json.dump(obj, f, indent=indent, default=default)
    else:
        f.write(str(obj))
    f.close()


# ------------------------------------------------------------------------------- tokenizers
class HashWordTokenizer:
    """Offline stand-in for an HF slow tokenizer (``use_fast=False``): words and punctuation map
    to stable ids by hashing into the non-special id range. Exposes the subset of the
    ``PreTrainedTokenizer`` API the SFT path uses."""

    _pat = re.compile(r"\w+|[^\w\s]|\n")

    def __init__(self, vocab_size: int, model_max_length: int = 512, pad_token: Optional[str] = None,
                 eos_token: Optional[str] = "</s>", bos_token: Optional[str] = "<s>",
                 unk_token: Optional[str] = "<unk>", special_ids: Optional[Dict[str, int]] = None,
                 padding_side: str = "right", add_bos_token: bool = True):
        self.base_vocab = int(vocab_size)
        self.add_bos_token = add_bos_token
        self.model_max_length = int(model_max_length)
        self.padding_side = padding_side
        self.added: Dict[str, int] = {}
        self.special: Dict[str, int] = dict(special_ids or {})
        self._tokens = {"pad_token": pad_token, "eos_token": eos_token, "bos_token": bos_token,
                        "unk_token": unk_token}
        nxt = 0
        for name, tok in self._tokens.items():
            if tok is not None and tok not in self.special:
                while nxt in self.special.values():
                    nxt += 1
                self.special[tok] = nxt
        self.first_free = max(self.special.values(), default=-1) + 1
        self.name_or_path = "hash-word"

    # token attributes like HF
    def __getattr__(self, k):
        if k.endswith("_token") and k in self.__dict__.get("_tokens", {}):
            return self._tokens[k]
        if k.endswith("_token_id"):
            t = self.__dict__["_tokens"].get(k[:-3])
            return None if t is None else self.convert_tokens_to_ids(t)
        raise AttributeError(k)

    def __len__(self):
        return self.base_vocab + len(self.added)

    def convert_tokens_to_ids(self, tok):
        if tok in self.added:
            return self.added[tok]
        return self.special.get(tok, self.special.get(self._tokens.get("unk_token") or "", 0))

    def add_special_tokens(self, d: Dict[str, str]) -> int:
        n = 0
        for name, tok in d.items():
            self._tokens[name] = tok
            if tok not in self.special and tok not in self.added:
                self.added[tok] = len(self)
                n += 1
        return n

    def _piece_id(self, piece: str) -> int:
        if piece in self.special:
            return self.special[piece]
        if piece in self.added:
            return self.added[piece]
        h = int.from_bytes(hashlib.blake2b(piece.encode(), digest_size=8).digest(), "little")
        return self.first_free + h % (self.base_vocab - self.first_free)

    def encode(self, text: str) -> List[int]:
        out: List[int] = []
        specials = sorted([t for t in list(self.special) + list(self.added) if t], key=len, reverse=True)
        if specials:
            parts = re.split("(" + "|".join(re.escape(t) for t in specials) + ")", text)
        else:
            parts = [text]
        for p in parts:
            if not p:
                continue
            if p in self.special or p in self.added:
                out.append(self._piece_id(p))
            else:
                out.extend(self._piece_id(w) for w in self._pat.findall(p))
        return out

    def __call__(self, text, return_tensors=None, padding=None, max_length=None, truncation=False, **_):
        ids = self.encode(text)
        if self.add_bos_token and self._tokens.get("bos_token"):
            ids = [self.convert_tokens_to_ids(self._tokens["bos_token"])] + ids
        if truncation:
            ids = ids[: (max_length or self.model_max_length)]
        if return_tensors == "pt":
            return _Enc(torch.tensor([ids], dtype=torch.long))
        return {"input_ids": ids}

    def save_pretrained(self, d):
        os.makedirs(d, exist_ok=True)
        jdump({"tokenizer_class": "HashWordTokenizer", "vocab_size": self.base_vocab, "added": self.added,
               "special": self.special, "tokens": self._tokens, "model_max_length": self.model_max_length,
               "add_bos_token": self.add_bos_token},
              os.path.join(d, "smdt_tokenizer.json"))


class _Enc:
    def __init__(self, ids):
        self.input_ids = ids


OFFLINE_TOKENIZERS = {
    # name: (len(tokenizer), pad, eos, bos, unk, ids) — sizes/specials of the public tokenizers
    "opt": (50265, "<pad>", "</s>", "</s>", "<unk>", {"<s>": 0, "<pad>": 1, "</s>": 2, "<unk>": 3}),
    "llama": (32000, None, "</s>", "<s>", "<unk>", {"<unk>": 0, "<s>": 1, "</s>": 2}),
    "gpt2": (50257, None, "<|endoftext|>", "<|endoftext|>", "<|endoftext|>", {"<|endoftext|>": 50256}),
}


def load_tokenizer(name_or_path: str, cache_dir: Optional[str] = None, model_max_length: int = 512,
                   model_type: Optional[str] = None, padding_side: str = "right"):
    """``AutoTokenizer.from_pretrained(..., use_fast=False, padding_side='right')`` when the files
    exist locally (``name_or_path`` dir or ``cache_dir/name_or_path``); otherwise the offline
    ``HashWordTokenizer`` with the same vocab size and special ids."""
    cands = [name_or_path] + ([os.path.join(cache_dir, name_or_path)] if cache_dir else [])
    for c in cands:
        if os.path.isdir(c) and any(os.path.exists(os.path.join(c, f)) for f in
                                    ("tokenizer_config.json", "vocab.json", "tokenizer.model", "tokenizer.json")):
            import transformers
            return transformers.AutoTokenizer.from_pretrained(c, model_max_length=model_max_length,
                                                              padding_side=padding_side, use_fast=False)
        if os.path.exists(os.path.join(c, "smdt_tokenizer.json")):
            d = jload(os.path.join(c, "smdt_tokenizer.json"))
            t = HashWordTokenizer(d["vocab_size"], model_max_length, special_ids=d["special"],
                                  padding_side=padding_side, add_bos_token=d.get("add_bos_token", True),
                                  **{k: v for k, v in d["tokens"].items()})
            t.added = {k: int(v) for k, v in d["added"].items()}
            return t
    mt = model_type
    if mt is None:
        low = name_or_path.lower()
        mt = "opt" if "opt" in low else "llama" if "llama" in low else "gpt2"
    n, pad, eos, bos, unk, ids = OFFLINE_TOKENIZERS[mt]
    log.warning("no local tokenizer files for %s: using the offline HashWordTokenizer (%d ids)", name_or_path, n)
    return HashWordTokenizer(n, model_max_length, pad, eos, bos, unk, ids, padding_side, add_bos_token=mt != "gpt2")


# ------------------------------------------------------------------------------- preprocessing
def _tokenize_fn(strings: Sequence[str], tokenizer) -> Dict:
    ids = []
    for text in strings:
        t = tokenizer(text, return_tensors="pt", padding="longest", max_length=tokenizer.model_max_length,
                      truncation=True)
        ids.append(t.input_ids[0])
    pad = tokenizer.pad_token_id
    lens = [int(x.ne(pad).sum().item()) if pad is not None else len(x) for x in ids]
    return dict(input_ids=ids, labels=ids, input_ids_lens=lens, labels_lens=lens)


def preprocess(sources: Sequence[str], targets: Sequence[str], tokenizer) -> Dict:
    """Tokenise source+target; mask the source part of the labels with ``IGNORE_INDEX``."""
    examples = [s + t for s, t in zip(sources, targets)]
    ex_tok = _tokenize_fn(examples, tokenizer)
    src_tok = _tokenize_fn(sources, tokenizer)
    input_ids = ex_tok["input_ids"]
    labels = [x.clone() for x in input_ids]
    for lab, n in zip(labels, src_tok["input_ids_lens"]):
        lab[:n] = IGNORE_INDEX
    return dict(input_ids=input_ids, labels=labels)


def format_examples(list_data_dict, eos_token: str):
    pi, pn = PROMPT_DICT["prompt_input"], PROMPT_DICT["prompt_no_input"]
    sources = [pi.format_map(e) if e.get("input", "") != "" else pn.format_map(e) for e in list_data_dict]
    targets = [f"{e['output']}{eos_token}" for e in list_data_dict]
    return sources, targets


class SupervisedDataset(Dataset):
    """Alpaca SFT dataset; stores token ids as one flat int32 array + offsets."""

    def __init__(self, data_path: str, tokenizer, cache_dir: Optional[str] = None):
        super().__init__()
        cache = None
        if cache_dir:
            key = hashlib.md5(f"{os.path.abspath(data_path)}:{os.path.getsize(data_path)}:"
                              f"{os.path.getmtime(data_path)}:{len(tokenizer)}:{tokenizer.model_max_length}:"
                              f"{getattr(tokenizer, 'name_or_path', '')}".encode()).hexdigest()
            cache = os.path.join(cache_dir, f"sft_{key}.npz")
        if cache and os.path.exists(cache):
            z = np.load(cache)
            self.ids, self.lab, self.off = z["ids"], z["lab"], z["off"]
            return
        log.warning("Loading data...")
        data = jload(data_path)
        log.warning("Formatting inputs...")
        sources, targets = format_examples(data, tokenizer.eos_token)
        log.warning("Tokenizing inputs... This may take some time...")
        d = preprocess(sources, targets, tokenizer)
        lens = np.array([len(x) for x in d["input_ids"]], dtype=np.int64)
        self.off = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
        self.ids = torch.cat(d["input_ids"]).to(torch.int32).numpy() if len(lens) else np.zeros(0, np.int32)
        self.lab = torch.cat(d["labels"]).to(torch.int32).numpy() if len(lens) else np.zeros(0, np.int32)
        if cache:
            os.makedirs(cache_dir, exist_ok=True)
            tmp = cache + f".tmp{os.getpid()}.npz"
            np.savez(tmp, ids=self.ids, lab=self.lab, off=self.off)
            os.replace(tmp, cache)

    def __len__(self):
        return len(self.off) - 1

    def lengths(self) -> np.ndarray:
        return np.diff(self.off)

    def __getitem__(self, i) -> Dict[str, torch.Tensor]:
        s, e = int(self.off[i]), int(self.off[i + 1])
        return dict(input_ids=torch.from_numpy(self.ids[s:e].astype(np.int64)),
                    labels=torch.from_numpy(self.lab[s:e].astype(np.int64)))


@dataclass
class DataCollatorForSupervisedDataset:
    """Right-pad ids (pad id) and labels (-100); ``pad_to_multiple_of`` rounds the batch length up."""

    tokenizer: object
    pad_to_multiple_of: int = 1

    def __call__(self, instances: Sequence[Dict]) -> Dict[str, torch.Tensor]:
        ids = [x["input_ids"] for x in instances]
        labs = [x["labels"] for x in instances]
        L = max(len(x) for x in ids)
        m = max(1, int(self.pad_to_multiple_of))
        L = ((L + m - 1) // m) * m
        pad = self.tokenizer.pad_token_id
        out_ids = torch.full((len(ids), L), pad, dtype=torch.long)
        out_lab = torch.full((len(ids), L), IGNORE_INDEX, dtype=torch.long)
        for i, (a, b) in enumerate(zip(ids, labs)):
            out_ids[i, : len(a)] = a
            out_lab[i, : len(b)] = b
        return dict(input_ids=out_ids, labels=out_lab, attention_mask=out_ids.ne(pad))


def make_supervised_data_module(tokenizer, data_args, cache_dir: Optional[str] = None,
                                pad_to_multiple_of: int = 1) -> Dict:
    ds = SupervisedDataset(data_args.data_path, tokenizer, cache_dir=cache_dir)
    return dict(train_dataset=ds, eval_dataset=None,
                data_collator=DataCollatorForSupervisedDataset(tokenizer, pad_to_multiple_of))


# ------------------------------------------------------------------------------- samplers
class DistributedRandomSampler(Sampler):
    """Per-epoch seeded permutation, split round-robin over ranks (drop nothing, pad by wrap)."""

    def __init__(self, n: int, rank: int = 0, world: int = 1, seed: int = 42, shuffle: bool = True):
        self.n, self.rank, self.world, self.seed, self.shuffle = n, rank, world, seed, shuffle
        self.epoch = 0
        self.num_samples = (n + world - 1) // world

    def set_epoch(self, e):
        self.epoch = e

    def _order(self):
        if self.shuffle:
            g = torch.Generator().manual_seed(self.seed + self.epoch)
            return torch.randperm(self.n, generator=g).tolist()
        return list(range(self.n))

    def __iter__(self):
        idx = self._order()
        total = self.num_samples * self.world
        idx = (idx * ((total + len(idx) - 1) // max(len(idx), 1)))[:total]
        return iter(idx[self.rank:total:self.world])

    def __len__(self):
        return self.num_samples


class LengthGroupedSampler(DistributedRandomSampler):
    """HF ``group_by_length``: shuffle, cut into mega-batches of 50×(mbs×world), sort each by
    length (longest first) — batches of similar length waste less padding."""

    def __init__(self, lengths, batch_size: int, rank=0, world=1, seed=42):
        super().__init__(len(lengths), rank, world, seed, True)
        self.lengths = np.asarray(lengths)
        self.batch_size = batch_size

    def _order(self):
        idx = super()._order()
        mb = self.batch_size * self.world * 50
        out = []
        for i in range(0, len(idx), mb):
            chunk = idx[i:i + mb]
            chunk.sort(key=lambda j: -int(self.lengths[j]))
            out.extend(chunk)
        # __iter__ deals positions round-robin, so rank r's micro-batch k takes sorted positions
        # k*mbs*world + j*world + r: every rank's k-th batch comes from the same sorted window.
        return out


# ------------------------------------------------------------------------------- synthetic data
_WORDS = ("the of and to in is that for it as with was on be by this are or from at an which have not "
          "data model write explain describe list give create generate summarize translate classify "
          "sentence paragraph story poem function code number answer question example words following "
          "time people world water energy system process plan idea city country language music").split()


def write_synthetic_alpaca(path: str, n: int = 52002, seed: int = 0):
    """Alpaca-shaped synthetic JSON. Word counts follow the public Alpaca-52K set (instruction ~ 13
    words, input present 40 % ~ 10 words, output ~ 45 words with a long tail), scaled by 1.3 —
    the BPE tokens per English word of the GPT-2 / LLaMA tokenizers — because the offline
    tokenizer maps one word to one id. With the prompt template that gives ~125 tokens per example
    (median ~110, p99 ~360, 0.3 % cut by the ``model_max_length`` 512 cap), like the
    real set under the reference's tokenizer (/root/reference/4_training_alpaca_deepspeed/
    train.py:86-89)."""
    rng = random.Random(seed)

    def sent(k):
        return " ".join(rng.choice(_WORDS) for _ in range(max(1, k))).capitalize() + "."

    data = []
    for _ in range(n):
        ins = sent(int(1.3 * rng.gauss(13, 5)))
        inp = sent(int(1.3 * rng.expovariate(1 / 10))) if rng.random() < 0.4 else ""
        out = sent(int(1.3 * min(rng.lognormvariate(3.5, 0.8), 600)))
        data.append({"instruction": ins, "input": inp, "output": out})
    jdump(data, path)
    return path
