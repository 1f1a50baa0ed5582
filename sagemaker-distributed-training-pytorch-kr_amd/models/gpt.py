"""GPT model (Megatron ``GPTModel`` semantics) for pipeline / tensor / sequence parallelism.

Reference behaviour: `model_provider` builds
``GPTModel(config, num_tokentypes=0, parallel_output=True, pre_process, post_process)``
(/root/reference/3_training_megatron-lm/pretrain_gpt.py:46-58); with labels the model returns the
per-token LM loss [b, s] computed by the vocab-parallel cross entropy; vocab is padded to a
multiple of ``make_vocab_size_divisible_by * tp`` (NB3:1212); word embeddings are tied to the
output layer unless ``--untie-embeddings-and-output-weights``.
"""
from __future__ import annotations

import math
from typing import Optional

import torch
import torch.distributed as dist
import torch.nn as nn

from ..ops import functional as SF
from ..parallel import state as ps
from ..parallel import tensor_parallel as tp
from .transformer import ParallelTransformer, TransformerConfig


def pad_vocab_size(orig: int, divisible_by: int = 128, tp_size: int = 1) -> int:
    """Megatron's ``_vocab_size_with_padding``."""
    m = divisible_by * tp_size
    return ((orig + m - 1) // m) * m


def stage_layer_range(num_layers: int, pp: int, pp_rank: int, vpp: Optional[int] = None, vpp_rank: int = 0,
                      first: Optional[int] = None, last: Optional[int] = None):
    """(first_layer, count) for a (virtual) pipeline stage. Layers split uniformly, except that
    ``first`` / ``last`` (Megatron-core ``--decoder-first/last-pipeline-num-layers``) fix the
    first / last stage's count and the middle stages share the rest evenly."""
    if vpp is None and pp > 1 and (first is not None or last is not None):
        counts = [None] * pp
        if first is not None:
            counts[0] = int(first)
        if last is not None:
            counts[-1] = int(last)
        rest = num_layers - sum(c for c in counts if c is not None)
        free = [i for i, c in enumerate(counts) if c is None]
        if rest < 0 or (free and rest % len(free)) or (not free and rest != 0):
            raise ValueError(f"cannot split {num_layers} layers over {pp} stages with first={first} last={last}")
        for i in free:
            counts[i] = rest // len(free)
        return sum(counts[:pp_rank]), counts[pp_rank]
    if vpp is None:
        assert num_layers % pp == 0, "num_layers must be divisible by the pipeline size"
        n = num_layers // pp
        return pp_rank * n, n
    assert first is None and last is None, "uneven pipeline splits are not supported with virtual stages"
    assert num_layers % (pp * vpp) == 0
    n = num_layers // (pp * vpp)
    return vpp_rank * (num_layers // vpp) + pp_rank * n, n


class GPTModel(nn.Module):
    def __init__(self, cfg: TransformerConfig, pre_process: bool = True, post_process: bool = True,
                 parallel_output: bool = True, device=None, layer_range=None):
        super().__init__()
        with tp.weight_init(cfg.init_method, cfg.perform_initialization, cfg.use_cpu_initialization):
            self._build(cfg, pre_process, post_process, parallel_output, device, layer_range)

    def _build(self, cfg, pre_process, post_process, parallel_output, device, layer_range):
        st = ps.get_state()
        self.cfg = cfg
        self.pre_process, self.post_process = pre_process, post_process
        self.parallel_output = parallel_output
        self.sp = cfg.sequence_parallel and st.tp > 1
        if layer_range is None:
            layer_range = stage_layer_range(cfg.num_layers, st.pp, st.pp_rank, st.virtual_pp, st.virtual_pp_rank,
                                            cfg.decoder_first_pipeline_num_layers,
                                            cfg.decoder_last_pipeline_num_layers)
        first, n = layer_range
        self.first_layer, self.num_local_layers = first, n
        std = cfg.init_method_std
        if pre_process:
            self.embedding = tp.VocabParallelEmbedding(cfg.padded_vocab_size, cfg.hidden_size, init_std=std,
                                                       key="embedding.word", seed=cfg.seed,
                                                       params_dtype=cfg.params_dtype, device=device)
            if cfg.position_embedding_type == "learned_absolute":
                w = tp.init_full_then_shard((cfg.max_position_embeddings + cfg.position_offset, cfg.hidden_size), std,
                                            "embedding.position.weight", cfg.seed, cfg.params_dtype, device, None, 0, 1)
                self.position_embeddings = nn.Parameter(w)
            else:
                self.position_embeddings = None
        self.decoder = ParallelTransformer(cfg, first, n, post_norm=post_process, device=device)
        self.output_weight = None
        if post_process:
            if cfg.untie_embeddings_and_output_weights:
                w = tp.init_full_then_shard((cfg.padded_vocab_size, cfg.hidden_size), std, "output_layer.weight",
                                            cfg.seed, cfg.params_dtype, device, 0, st.tp_rank, st.tp)
                self.output_weight = nn.Parameter(w)
                self.output_weight.tensor_model_parallel = True
            elif not pre_process:
                # Tied embeddings across pipeline stages: the last stage keeps its own copy,
                # initialised identically and kept in sync by an embedding-group all-reduce of
                # the gradients (`allreduce_word_embedding_grads`).
                w = tp.init_full_then_shard((cfg.padded_vocab_size, cfg.hidden_size), std, "embedding.word.weight",
                                            cfg.seed, cfg.params_dtype, device, 0, st.tp_rank, st.tp)
                self.output_weight = nn.Parameter(w)
                self.output_weight.tensor_model_parallel = True
                self.output_weight.shared_embedding = True
        if pre_process and post_process is False and not cfg.untie_embeddings_and_output_weights and st.pp > 1:
            self.embedding.weight.shared_embedding = True
        if pre_process and post_process and not cfg.untie_embeddings_and_output_weights:
            # tied LM head on the same stage: the weight receives its gradient twice (fused wgrad
            # into main_grad + the lookup's autograd accumulation)
            self.embedding.weight._smdt_grad_contributions = 2
        self.input_tensor = None
        # > 0: logits columns >= this are vocab padding and are excluded from the loss (HF models)
        self.loss_vocab_size = 0
        if cfg.position_embedding_type == "rope":
            rot = int(cfg.kv_channels * cfg.rotary_percent)
            rot -= rot % 16
            cos, sin = SF.rope_tables(cfg.max_position_embeddings, rot, cfg.rotary_base, device=device)
            self.register_buffer("rope_cos", cos, persistent=False)
            self.register_buffer("rope_sin", sin, persistent=False)
            for layer in self.decoder.layers:
                layer.attention.set_rope(self.rope_cos, self.rope_sin, rot)

    # ---- pipeline plumbing
    def set_input_tensor(self, t):
        self.input_tensor = t

    def word_embeddings_weight(self):
        if self.pre_process:
            return self.embedding.weight
        return self.output_weight

    def _embed(self, tokens, position_ids, pos_start=None):
        """[s, b, h] embeddings. ``pos_start`` (int): positions are pos_start + arange(s) in every
        sequence, so the position table is a slice broadcast over the batch (no gather, and a
        batch-sum backward instead of a [s * b]-row scatter)."""
        st = ps.get_state()
        e = self.embedding(tokens.t(), reduce=False)              # [s, b, h] (TP-partial), no transpose copy
        if st.tp > 1:
            if self.sp:
                e = tp.reduce_scatter_to_sequence_parallel_region(e)
            else:
                e = tp.reduce_from_tensor_model_parallel_region(e)
        if self.position_embeddings is not None and pos_start is not None and not self.sp:
            e = tp.add_position_slice(e, self.position_embeddings, pos_start + self.cfg.position_offset)
        elif self.position_embeddings is not None:
            pos = position_ids.transpose(0, 1)                   # [s, b]
            if self.cfg.position_offset:
                pos = pos + self.cfg.position_offset
            pe = tp.embedding_lookup(pos, self.position_embeddings)  # [s, b, h]
            if self.sp:
                pe = tp.scatter_to_sequence_parallel_region(pe)
            e = e + pe
        return e

    def lm_logits(self, h):
        st = ps.get_state()
        w = self.output_weight if self.output_weight is not None else self.embedding.weight
        logits = tp.linear_with_grad_accumulation_and_async_allreduce(
            h, w, None, sequence_parallel=self.sp, async_grad_allreduce=(st.tp > 1 and not self.sp))
        if not self.parallel_output:
            logits = tp.gather_from_tensor_model_parallel_region(logits)
        return logits                                            # [s, b, V / tp]

    def forward(self, tokens, position_ids=None, attention_mask=None, labels=None, loss_mask=None):
        """Returns per-token losses [b, s] when ``labels`` are given, else the logits. ``loss_mask``
        is accepted for Megatron's forward_step signature; the caller applies it to the losses."""
        if self.pre_process:
            pos_start = getattr(position_ids, "_smdt_arange_start", None) if position_ids is not None else None
            if position_ids is None:
                # with context parallelism ``tokens`` is this rank's chunk cp_rank of the sequence
                off = ps.get_state().cp_rank * tokens.shape[1]
                pos_start = off
                position_ids = (torch.arange(tokens.shape[1], device=tokens.device) + off).unsqueeze(0).expand_as(tokens)
            x = self._embed(tokens, position_ids, pos_start)
        else:
            x = self.input_tensor
        out = self.decoder(x, None, None)
        if not self.post_process:
            px, pb, res = out
            return SF.bias_dropout_add(px, pb, res, self.cfg.hidden_dropout, self.training)
        st = ps.get_state()
        if labels is not None:
            w = self.output_weight if self.output_weight is not None else self.embedding.weight
            if tp.lm_head_ce_ok(out, w, st.tp):
                # LM-head GEMM + CE as one op: no backward pass over the [tokens, vocab] logits
                vs = int(self.loss_vocab_size or 0)
                vvalid = vs if 0 < vs < w.shape[0] else 0
                loss = tp.LMHeadCrossEntropy.apply(out, w, labels.transpose(0, 1), -100, vvalid)
                return loss.transpose(0, 1).contiguous()             # [b, s]
            if self.parallel_output and tp.vp_lm_head_ce_ok(out, w, st.tp):
                # vocab-parallel LM head + CE as one op: one pass over this rank's logit slice
                vl = w.shape[0]
                vstart = st.tp_rank * vl
                vs = int(self.loss_vocab_size or 0)
                vvalid = min(max(vs - vstart, 0), vl) if vs > 0 else 0
                assert vs <= 0 or vvalid > 0, "a vocab shard holds only padding; use a smaller padding multiple"
                loss = tp.VocabParallelLMHeadCE.apply(out, w, labels.transpose(0, 1), -100, vstart,
                                                      0 if vvalid == vl else vvalid, bool(self.sp))
                return loss.transpose(0, 1).contiguous()             # [b, s]
        logits = self.lm_logits(out)
        if labels is None:
            return logits.transpose(0, 1).contiguous()
        vstart = st.tp_rank * (self.cfg.padded_vocab_size // st.tp) if self.parallel_output else 0
        group = st.tp_group if (st.tp > 1 and self.parallel_output) else None
        loss = SF.cross_entropy(logits, labels.transpose(0, 1), vstart, group, inplace_grad=True,
                                vocab_size=self.loss_vocab_size)
        return loss.transpose(0, 1).contiguous()                 # [b, s]


def allreduce_word_embedding_grads(model: GPTModel):
    """Sum tied word-embedding grads between the first and last pipeline stage (Megatron's
    embedding group)."""
    st = ps.get_state()
    if isinstance(model, nn.ModuleList):  # interleaved pipeline chunks
        if st.is_first_stage(ignore_virtual=True):
            model = model[0]
        elif st.is_last_stage(ignore_virtual=True):
            model = model[-1]
        else:
            return
    if st.pp == 1 or model.cfg.untie_embeddings_and_output_weights or st.embd_group is None:
        return
    if not (st.is_first_stage(ignore_virtual=True) or st.is_last_stage(ignore_virtual=True)):
        return
    w = model.word_embeddings_weight()
    g = getattr(w, "main_grad", None)
    if g is None:
        g = w.grad
    if g is not None:
        from ..comm import stats as _cs
        with _cs.blocking("all_reduce", st.embd_group, g.numel() * g.element_size()):
            dist.all_reduce(g, group=st.embd_group)


def gpt_flops_per_token(cfg: TransformerConfig, seq_len: int, recompute: bool = False) -> float:
    """Model FLOPs per token, Megatron's formula 72 B s L h^2 (1 + s/6h + V/12Lh) / (B s)
    (x 4/3 with full recompute); the reference's 41 TFLOP/s/GPU is derived with it."""
    L, h, V = cfg.num_layers, cfg.hidden_size, cfg.padded_vocab_size
    f = 72.0 * L * h * h * (1.0 + seq_len / (6.0 * h) + V / (12.0 * L * h))
    if cfg.activation == "swiglu" or cfg.num_query_groups != cfg.num_attention_heads:
        # exact count for non-GPT2 shapes: 6 * (params in matmuls) + attention
        hd = cfg.kv_channels
        qkv = h * (cfg.num_attention_heads + 2 * cfg.num_query_groups) * hd
        proj = cfg.num_attention_heads * hd * h
        ff = h * cfg.ffn_hidden_size * (3 if cfg.activation == "swiglu" else 2)
        per_layer = 6 * (qkv + proj + ff) + 12 * seq_len * cfg.num_attention_heads * hd
        f = L * per_layer + 6 * h * V
    return f * (4.0 / 3.0 if recompute else 1.0)


GPT_CONFIGS = {
    # name: (layers, hidden, heads, seq)
    "gpt2-small": dict(num_layers=12, hidden_size=768, num_attention_heads=12),
    "gpt2-medium": dict(num_layers=24, hidden_size=1024, num_attention_heads=16),   # "345M"
    "gpt2-345m": dict(num_layers=24, hidden_size=1024, num_attention_heads=16),
    "gpt3-1.3b": dict(num_layers=24, hidden_size=2048, num_attention_heads=16),
    "gpt3-6.7b": dict(num_layers=32, hidden_size=4096, num_attention_heads=32),
    "llama-7b": dict(num_layers=32, hidden_size=4096, num_attention_heads=32, activation="swiglu",
                     normalization="RMSNorm", position_embedding_type="rope", add_bias_linear=False,
                     ffn_hidden_size=11008, layernorm_epsilon=1e-6, untie_embeddings_and_output_weights=True),
}
