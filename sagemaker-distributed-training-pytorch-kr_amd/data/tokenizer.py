"""Tokenizers for the GPT recipe.

``GPT2BPETokenizer`` is the reference default (`args_defaults={'tokenizer_type':
'GPT2BPETokenizer'}`, /root/reference/3_training_megatron-lm/pretrain_gpt.py:149) built from
``--vocab-file`` / ``--merge-file``; it wraps the local ``transformers`` GPT-2 BPE implementation
(no network: files must exist). ``NullTokenizer`` serves synthetic / pre-tokenised data.
``vocab_size_with_padding`` reproduces Megatron's padding (50,257 -> 50,688 at TP=4 with
divisible-by 128, NB3:1212).
"""
from __future__ import annotations

from typing import List


def vocab_size_with_padding(orig_vocab_size: int, make_vocab_size_divisible_by: int = 128, tp: int = 1) -> int:
    m = make_vocab_size_divisible_by * tp
    return ((orig_vocab_size + m - 1) // m) * m


class AbstractTokenizer:
    name = "abstract"

    @property
    def vocab_size(self) -> int:
        raise NotImplementedError

    def tokenize(self, text: str) -> List[int]:
        raise NotImplementedError

    def detokenize(self, ids) -> str:
        raise NotImplementedError

    @property
    def eod(self) -> int:
        raise NotImplementedError


class GPT2BPETokenizer(AbstractTokenizer):
    name = "GPT2BPETokenizer"

    def __init__(self, vocab_file: str, merge_file: str):
        import inspect
        import json
        from transformers import GPT2Tokenizer
        with open(vocab_file, encoding="utf-8") as f:
            self.encoder = json.load(f)
        params = inspect.signature(GPT2Tokenizer.__init__).parameters
        if "vocab" in params:   # transformers >= 5: the tokenizers-backed class takes the data itself
            with open(merge_file, encoding="utf-8") as f:
                merges = [tuple(ln.split()) for ln in f.read().split("\n")
                          if ln and not ln.startswith("#version") and len(ln.split()) == 2]
            self.tok = GPT2Tokenizer(vocab=self.encoder, merges=merges, errors="replace")
        else:
            self.tok = GPT2Tokenizer(vocab_file=vocab_file, merges_file=merge_file, errors="replace")
        self.eod_id = self.encoder.get("<|endoftext|>", self.tok.convert_tokens_to_ids("<|endoftext|>"))

    @property
    def vocab_size(self):
        return len(self.encoder)   # Megatron: len(encoder) of vocab.json (50,257 for GPT-2)

    def tokenize(self, text):
        return self.tok.encode(text)

    def detokenize(self, ids):
        return self.tok.decode(list(ids))

    @property
    def eod(self):
        return self.eod_id


class HFTokenizer(AbstractTokenizer):
    """Any local HuggingFace tokenizer directory (``--tokenizer-model``)."""
    name = "HuggingFaceTokenizer"

    def __init__(self, path: str, **kw):
        from transformers import AutoTokenizer
        self.tok = AutoTokenizer.from_pretrained(path, local_files_only=True, **kw)

    @property
    def vocab_size(self):
        return len(self.tok)

    def tokenize(self, text):
        return self.tok.encode(text, add_special_tokens=False)

    def detokenize(self, ids):
        return self.tok.decode(list(ids))

    @property
    def eod(self):
        return self.tok.eos_token_id


class NullTokenizer(AbstractTokenizer):
    """Identity tokenizer over whitespace-separated ids; EOD = vocab_size - 1."""
    name = "NullTokenizer"

    def __init__(self, vocab_size: int):
        self._v = int(vocab_size)

    @property
    def vocab_size(self):
        return self._v

    def tokenize(self, text):
        return [int(t) for t in text.split()]

    def detokenize(self, ids):
        return " ".join(str(int(i)) for i in ids)

    @property
    def eod(self):
        return self._v - 1


def build_tokenizer(tokenizer_type: str, vocab_file=None, merge_file=None, tokenizer_model=None, vocab_size=None,
                    make_vocab_size_divisible_by=128, tensor_model_parallel_size=1, rank=0):
    """Returns (tokenizer, padded_vocab_size)."""
    if tokenizer_type == "GPT2BPETokenizer":
        if not (vocab_file and merge_file):
            raise ValueError("GPT2BPETokenizer needs --vocab-file and --merge-file")
        tok = GPT2BPETokenizer(vocab_file, merge_file)
    elif tokenizer_type in ("HuggingFaceTokenizer", "HFTokenizer"):
        tok = HFTokenizer(tokenizer_model)
    elif tokenizer_type == "NullTokenizer":
        tok = NullTokenizer(vocab_size or 50257)
    else:
        raise ValueError(f"unsupported tokenizer {tokenizer_type}")
    padded = vocab_size_with_padding(tok.vocab_size, make_vocab_size_divisible_by, tensor_model_parallel_size)
    if rank == 0:
        print(f" > padded vocab (size: {tok.vocab_size}) with {padded - tok.vocab_size} dummy tokens "
              f"(new size: {padded})", flush=True)
    return tok, padded
