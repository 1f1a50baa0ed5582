"""Megatron-compatible parallel transformer (GPT / LLaMA families) on the gfx950 kernel library.

Covers the model side of the reference's Megatron recipe (`core_transformer_config_
from_args`, /root/reference/3_training_megatron-lm/megatron/arguments.py:419-446, GPTModel at
`pretrain_gpt.py:46-58`): pre-LN blocks, learned-absolute or RoPE positions, GeLU / SwiGLU /
squared-ReLU MLPs, MHA or GQA, hidden/attention dropout, TP + SP + activation recompute.

Activation layout is [s, b, h] (sequence-first, as Megatron) so sequence-parallel shards are
contiguous chunks and the TP collectives move contiguous buffers.

The residual stream is "deferred": a layer returns (branch_output, branch_bias) plus the
residual, and the NEXT layer's first LayerNorm consumes them through ONE fused kernel
(bias + dropout + residual-add + LayerNorm, K4+K6), so the residual stream is written once and
read once per sub-block. Layer 0 folds the embedding dropout into the same kernel.
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass, field
from typing import Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops import _ext
from ..ops import functional as SF
from ..parallel import state as ps
from ..parallel import tensor_parallel as tp
from ..parallel.random import checkpoint as rng_checkpoint, get_rng


@dataclass
class TransformerConfig:
    num_layers: int = 24
    hidden_size: int = 1024
    num_attention_heads: int = 16
    num_query_groups: Optional[int] = None       # GQA (None -> MHA)
    ffn_hidden_size: Optional[int] = None        # default 4h (GeLU) / 8h/3 rounded (SwiGLU)
    kv_channels: Optional[int] = None
    # uneven pipeline split (Megatron-core --decoder-first/last-pipeline-num-layers): the last
    # stage also runs the LM head + CE, so giving it fewer layers balances the pipeline
    decoder_first_pipeline_num_layers: Optional[int] = None
    decoder_last_pipeline_num_layers: Optional[int] = None
    hidden_dropout: float = 0.1
    attention_dropout: float = 0.1
    layernorm_epsilon: float = 1e-5
    layernorm_zero_centered_gamma: bool = False  # --apply-layernorm-1p: gamma stored as (gamma - 1)
    apply_residual_connection_post_layernorm: bool = False   # residual taken after the norm
    normalization: str = "LayerNorm"            # or "RMSNorm"
    activation: str = "gelu"                     # gelu | swiglu | squared_relu | gelu_erf
    num_experts: Optional[int] = None            # --num-experts: Switch MLP (top-1 routed experts)
    add_bias_linear: bool = True
    position_embedding_type: str = "learned_absolute"   # or "rope"
    rotary_percent: float = 1.0
    rotary_base: float = 10000.0
    max_position_embeddings: int = 1024
    position_offset: int = 0                     # OPT's learned positions start at row 2
    padded_vocab_size: int = 50304
    untie_embeddings_and_output_weights: bool = False
    init_method_std: float = 0.02
    init_method: str = "normal"                  # or "xavier_uniform" (--init-method-xavier-uniform)
    perform_initialization: bool = True         # False: --no-initialization (weights left unset)
    use_cpu_initialization: bool = False        # --use-cpu-initialization: draw on the host
    params_dtype: torch.dtype = torch.bfloat16
    seed: int = 1234
    # parallelism
    sequence_parallel: bool = False
    async_tensor_model_parallel_allreduce: bool = True
    # fusions (Megatron --no-*-fusion flags turn these off)
    masked_softmax_fusion: bool = True
    bias_gelu_fusion: bool = True
    bias_dropout_fusion: bool = True
    use_flash_attn: bool = True
    apply_query_key_layer_scaling: bool = False
    # recompute (P9)
    recompute_granularity: Optional[str] = None  # "full" | "selective"
    recompute_method: Optional[str] = None       # "uniform" | "block"
    recompute_num_layers: Optional[int] = None
    distribute_saved_activations: bool = False   # full recompute: saved layer inputs split across TP

    def __post_init__(self):
        if self.num_query_groups is None:
            self.num_query_groups = self.num_attention_heads
        if self.kv_channels is None:
            self.kv_channels = self.hidden_size // self.num_attention_heads
        if self.ffn_hidden_size is None:
            if self.activation == "swiglu":
                f = int(8 * self.hidden_size / 3)
                self.ffn_hidden_size = 256 * ((f + 255) // 256)
            else:
                self.ffn_hidden_size = 4 * self.hidden_size

    @property
    def rms(self) -> bool:
        return self.normalization.lower() == "rmsnorm"


def _gather_wait(mod, x):
    """Run ``mod``'s overlapped-ZeRO parameter all-gather wait (a forward pre-hook installed by
    parallel/distributed.py) for a module whose weights are read without calling ``mod(x)``
    (Norm.fused, the fused MLP paths). Without it the kernel could read weights whose async
    all-gather is still in flight. The wait is idempotent."""
    for hook in tuple(mod._forward_pre_hooks.values()):
        if getattr(hook, "_smdt_gather_wait", False):
            hook(mod, (x,))


class Norm(nn.Module):
    """LayerNorm / RMSNorm parameters; the math runs in the fused BDA+norm kernel."""

    def __init__(self, h, cfg: TransformerConfig, device=None):
        super().__init__()
        self.rms = cfg.rms
        self.eps = cfg.layernorm_epsilon
        # Sequence-parallel activations are sharded across TP: draw their dropout masks from the
        # per-TP-rank stream; replicated activations use the TP-identical default stream.
        self.rng_kind = "tp" if cfg.sequence_parallel and ps.get_state().tp > 1 else "default"
        # --apply-layernorm-1p: the stored gamma is centred on zero (so weight decay pulls the
        # scale toward 1) and the kernel reads 1 + weight
        self.one_p = bool(cfg.layernorm_zero_centered_gamma)
        init = torch.zeros if self.one_p else torch.ones
        self.weight = nn.Parameter(init(h, dtype=cfg.params_dtype, device=device))
        self.weight.sequence_parallel = cfg.sequence_parallel
        if not self.rms:
            self.bias = nn.Parameter(torch.zeros(h, dtype=cfg.params_dtype, device=device))
            self.bias.sequence_parallel = cfg.sequence_parallel
        else:
            self.register_parameter("bias", None)

    def fused(self, x, xbias, residual, p, training, gather=None):
        # called instead of forward() by the layers: wait for this module's overlapped ZeRO
        # parameter all-gather (see _gather_wait) before the kernel reads the weights
        _gather_wait(self, x)
        w = self.weight + 1 if self.one_p else self.weight
        return SF.bias_dropout_add_norm(x, xbias, residual, w, self.bias, p, training, self.eps, self.rms,
                                        rng=get_rng(self.rng_kind), gather=gather)

    def forward(self, x):
        return self.fused(x, None, None, 0.0, False)[0]


# ---------------------------------------------------------------------------------------------
# Padding-free ("unpadded") micro-batches. An SFT micro-batch is right-padded to its longest
# example; with causal attention a real token never sees a pad, so the pads only cost compute.
# Under ``packed_sequences`` every token-wise op (embeddings, GEMMs, norms, MLP, LM head + CE)
# runs on the T real tokens only ([T, 1, h]); attention alone scatters its fused QKV into the
# padded [L, b] layout (zeros in the pad rows), runs RoPE + the causal flash kernels there and
# gathers the T context rows back. Real-token outputs and all gradients equal the padded
# computation's (models/hf.py ``HFCausalLM.forward`` sets it up from the attention mask).
_PACK = {"idx": None, "b": 0, "L": 0, "inv": None, "groups": None}


class packed_sequences:
    """Context: ``idx`` (device int64 [T]) = seq-first flat positions s * b + bi of the real
    tokens of a right-padded [b, L] batch. ``groups`` (optional, ``length_groups``): the rows
    bucketed by their own length, for the length-grouped attention layout."""

    def __init__(self, idx, b: int, L: int, groups=None):
        self.state = {"idx": idx, "b": int(b), "L": int(L), "inv": None, "groups": groups}

    def __enter__(self):
        self.prev = dict(_PACK)
        _PACK.update(self.state)
        return self

    def __exit__(self, *exc):
        _PACK.update(self.prev)
        return False


_PACK_GATHER = os.environ.get("SMDT_PACK_GATHER", "1") == "1"     # A/B: 0 = torch index ops


def _inv_map():
    """[L * b] int64: the packed row of each padded position, -1 for pads (cached per context)."""
    inv = _PACK.get("inv")
    if inv is None:
        idx, b, L = _PACK["idx"], _PACK["b"], _PACK["L"]
        inv = torch.full((L * b,), -1, dtype=torch.int64, device=idx.device)
        inv[idx] = torch.arange(idx.numel(), device=idx.device)
        _PACK["inv"] = inv
    return inv


class _GatherRows(torch.autograd.Function):
    """out[r] = x[fwd_map[r]] (0 where fwd_map[r] < 0); the gradient is the gather with
    ``bwd_map``, the inverse row map (ops: gather_rows in transpose.hip — every output row
    written once: no zero fill of the padded buffer, no index_copy / index_add scatter)."""

    @staticmethod
    def forward(ctx, x, fwd_map, bwd_map):
        ctx.bwd_map = bwd_map
        ctx.nin = x.shape[0]
        return _ext.ext().gather_rows(x.contiguous(), fwd_map)

    @staticmethod
    def backward(ctx, g):
        return _ext.ext().gather_rows(g.contiguous(), ctx.bwd_map), None, None


# Length-grouped attention layout (SMDT_SFT_LENGTH_GROUPS, default on). The padded [L, b] layout
# pays attention (and the row gathers) for every row at the window's longest length L: an NB4
# window of 32 Alpaca rows (~135 tokens each, the longest a few hundred) spends most of its causal
# attention on pad rows. Rows are instead bucketed by their own length rounded up to 128 (the
# flash kernels' S granularity) into blocks [L_g, b_g], laid out one after another in ONE
# [sum_g L_g b_g, W] buffer: ONE row gather in, the causal flash kernels per block on views of
# it (no copies either way), ONE gather out. Real-token results equal the [L, b] layout's: a real
# token still sees exactly its own row's earlier tokens.
_LENGTH_GROUPS = os.environ.get("SMDT_SFT_LENGTH_GROUPS", "1") in ("1", "force")   # force: skip the cost gate
_LENGTH_GROUPS_FORCE = os.environ.get("SMDT_SFT_LENGTH_GROUPS", "1") == "force"
_GROUP_ALIGN = 128


# When the grouping pays: the attention work it saves is ~7 x (b L^2 saved) x hidden FLOPs per
# layer (forward + backward, at ~150 TFLOP/s for the padded causal kernels at these lengths);
# each extra block costs per layer its own launches and host work, calibrated at 250 us from the
# two NB4 models: OPT-125m (hidden 768) ran 11 % slower grouped, LLaMA-7B (4096) 6-7 % faster
# (profiles/r5_sft_groups/).
_GROUP_LAUNCH_S = 250e-6
_GROUP_FLOPS = 1.5e14


def length_groups(mask_cpu, idx_cpu, device, hidden: int = None):
    """Host-side (CPU, no device sync) plan of the length-grouped layout for a right-padded
    [b, L] CPU ``mask_cpu`` whose packed tokens are the seq-first positions ``idx_cpu``:
    ``{"blocks": [(row offset, L_g, b_g)], "inv": [P] packed index of each grouped position
    (-1 = pad), "pack": [T] grouped position of each packed token (-1: a trailing pad token
    beyond its row's block, whose attention output is then 0)}``, the maps on ``device``. None
    when, for a model of this ``hidden`` size, the attention work saved would not pay for the
    extra launches."""
    b, L = mask_cpu.shape
    lens = mask_cpu.sum(1).clamp(min=1)
    Lr = ((lens + _GROUP_ALIGN - 1) // _GROUP_ALIGN) * _GROUP_ALIGN          # per-row block length
    blocks, off = [], 0
    row_off = torch.empty(b, dtype=torch.int64)      # block offset of each row's block
    row_j = torch.empty(b, dtype=torch.int64)        # the row's index inside its block
    row_b = torch.empty(b, dtype=torch.int64)        # rows in the row's block
    row_L = torch.empty(b, dtype=torch.int64)
    for Lg in sorted(set(Lr.tolist())):
        rows = (Lr == Lg).nonzero().squeeze(1)
        bg = rows.numel()
        blocks.append((off, int(Lg), int(bg)))
        row_off[rows] = off
        row_j[rows] = torch.arange(bg)
        row_b[rows] = bg
        row_L[rows] = Lg
        off += int(Lg) * bg
    if hidden is not None:
        saved = b * L * L - sum(bg * Lg * Lg for _, Lg, bg in blocks)
        if 7.0 * saved * hidden / _GROUP_FLOPS < (len(blocks) - 1) * _GROUP_LAUNCH_S:
            return None
    s_t, i_t = idx_cpu // b, idx_cpu % b
    ok = s_t < row_L[i_t]
    pos = row_off[i_t] + s_t * row_b[i_t] + row_j[i_t]
    pack = torch.where(ok, pos, torch.full_like(pos, -1))
    inv = torch.full((off,), -1, dtype=torch.int64)
    inv[pos[ok]] = torch.arange(idx_cpu.numel())[ok]
    return {"blocks": blocks, "inv": inv.to(device, non_blocking=True),
            "pack": pack.to(device, non_blocking=True), "rows": off}


class _RopeQKVGroups(torch.autograd.Function):
    """RoPE (in place) on the q / k parts of the length-grouped [P, W] buffer: one launch per
    block, positions (row // b_g) within the block."""

    @staticmethod
    def forward(ctx, x, cos, sin, rot, nh, nkv, hd, blocks):
        ctx.mark_dirty(x)
        for o, Lg, bg in blocks:
            _ext.ext().rope_(x[o:o + Lg * bg, :(nh + nkv) * hd].view(Lg * bg, nh + nkv, hd), cos, sin, rot,
                             bg, Lg, False)
        ctx.save_for_backward(cos, sin)
        ctx.cfg = (rot, nh, nkv, hd, blocks)
        return x

    @staticmethod
    def backward(ctx, g):
        cos, sin = ctx.saved_tensors
        rot, nh, nkv, hd, blocks = ctx.cfg
        d = g if g.is_contiguous() else g.contiguous()
        for o, Lg, bg in blocks:
            _ext.ext().rope_(d[o:o + Lg * bg, :(nh + nkv) * hd].view(Lg * bg, nh + nkv, hd), cos, sin, rot,
                             bg, Lg, True)
        return d, None, None, None, None, None, None, None


class _FlashQKVGroups(torch.autograd.Function):
    """Causal flash attention of every block [L_g, b_g] of the length-grouped [P, W] fused-QKV
    buffer, reading q / k / v as strided views of it and writing the context [P, nh hd] and, in
    backward, d(qkv) [P, W] block by block in place (the kernels take strided views)."""

    @staticmethod
    def forward(ctx, qkv, nh, nkv, hd, scale, dropout_p, seeds, blocks):
        C = _ext.ext()
        P, W = qkv.shape
        out = qkv.new_empty(P, nh, hd)
        lses = []
        for (o, Lg, bg), (seed, off) in zip(blocks, seeds):
            q, k, v = SF._qkv_views(qkv[o:o + Lg * bg].view(Lg, bg, W), nh, nkv, hd, True)
            ov = out[o:o + Lg * bg].view(Lg, bg, nh, hd).transpose(0, 1)
            lses.append(C.flash_fwd(q, k, v, scale, True, ov, dropout_p, seed, off)[1])
        ctx.save_for_backward(qkv, out, *lses)
        ctx.cfg = (nh, nkv, hd, scale, dropout_p, seeds, blocks)
        return out.view(P, nh * hd)

    @staticmethod
    def backward(ctx, dout):
        qkv, out, *lses = ctx.saved_tensors
        nh, nkv, hd, scale, dropout_p, seeds, blocks = ctx.cfg
        C = _ext.ext()
        P, W = qkv.shape
        dqkv = torch.empty_like(qkv)
        do_all = dout.contiguous().view(P, nh, hd)
        for (o, Lg, bg), (seed, off), lse in zip(blocks, seeds, lses):
            sl = slice(o, o + Lg * bg)
            q, k, v = SF._qkv_views(qkv[sl].view(Lg, bg, W), nh, nkv, hd, True)
            dq, dk, dv = SF._qkv_views(dqkv[sl].view(Lg, bg, W), nh, nkv, hd, True)
            o_v = out[sl].view(Lg, bg, nh, hd).transpose(0, 1)
            do_v = do_all[sl].view(Lg, bg, nh, hd).transpose(0, 1)
            C.flash_bwd(q, k, v, o_v, do_v, lse, scale, True, dq, dk, dv, dropout_p, seed, off)
        return dqkv, None, None, None, None, None, None, None


def _unpack_rows(x):
    """[T, 1, W] -> [L, b, W] with zero pad rows (differentiable)."""
    idx, b, L = _PACK["idx"], _PACK["b"], _PACK["L"]
    W = x.shape[-1]
    if _PACK_GATHER and _ext.use_kernels(x) and (W * x.element_size()) % 16 == 0:
        return _GatherRows.apply(x.reshape(-1, W), _inv_map(), idx).view(L, b, W)
    return x.new_zeros(L * b, W).index_copy(0, idx, x.reshape(-1, W)).view(L, b, W)


def _pack_rows(x):
    """[L, b, C] -> [T, 1, C] (the real-token rows)."""
    C = x.shape[-1]
    if _PACK_GATHER and _ext.use_kernels(x) and (C * x.element_size()) % 16 == 0:
        return _GatherRows.apply(x.reshape(-1, C), _PACK["idx"], _inv_map()).unsqueeze(1)
    return x.reshape(-1, C).index_select(0, _PACK["idx"]).unsqueeze(1)


class ParallelAttention(nn.Module):
    def __init__(self, cfg: TransformerConfig, layer_number: int, device=None):
        super().__init__()
        st = ps.get_state()
        self.cfg = cfg
        self.layer_number = layer_number
        tpn = st.tp
        assert cfg.num_attention_heads % tpn == 0 and cfg.num_query_groups % tpn == 0
        self.nh = cfg.num_attention_heads // tpn
        self.nkv = cfg.num_query_groups // tpn
        self.hd = cfg.kv_channels
        q_out = cfg.num_attention_heads * self.hd
        kv_out = cfg.num_query_groups * self.hd
        std = cfg.init_method_std
        out_std = std / math.sqrt(2.0 * cfg.num_layers)
        self.qkv = tp.ColumnParallelLinear(cfg.hidden_size, q_out + 2 * kv_out, bias=cfg.add_bias_linear,
                                           init_std=std, key=f"layers.{layer_number}.qkv", seed=cfg.seed,
                                           params_dtype=cfg.params_dtype, device=device,
                                           sequence_parallel=cfg.sequence_parallel,
                                           chunks=[q_out, kv_out, kv_out],
                                           async_tensor_model_parallel_allreduce=cfg.async_tensor_model_parallel_allreduce)
        self.proj = tp.RowParallelLinear(q_out, cfg.hidden_size, bias=cfg.add_bias_linear, init_std=out_std,
                                         key=f"layers.{layer_number}.proj", seed=cfg.seed,
                                         params_dtype=cfg.params_dtype, device=device,
                                         sequence_parallel=cfg.sequence_parallel, skip_bias_add=True)
        self.rope = None

    def set_rope(self, cos, sin, rot):
        self.rope = (cos, sin, rot)

    def core_attention_unfused(self, qkv, training):
        """Megatron's unfused path: baddbmm -> fused causal softmax (K1) -> dropout -> bmm."""
        s, b = qkv.shape[0], qkv.shape[1]
        q, k, v = SF._qkv_views(qkv, self.nh, self.nkv, self.hd, True)  # [b, s, h, d]
        if self.nkv != self.nh:
            rep = self.nh // self.nkv
            k = k.repeat_interleave(rep, dim=2)
            v = v.repeat_interleave(rep, dim=2)
        qh = q.permute(0, 2, 1, 3).reshape(b * self.nh, s, self.hd)
        kh = k.permute(0, 2, 3, 1).reshape(b * self.nh, self.hd, s)
        vh = v.permute(0, 2, 1, 3).reshape(b * self.nh, s, self.hd)
        scores = torch.bmm(qh, kh).view(b, self.nh, s, s)
        probs = SF.scaled_masked_softmax(scores, None, 1.0 / math.sqrt(self.hd), causal=True)
        if training and self.cfg.attention_dropout > 0:
            probs = F.dropout(probs, p=self.cfg.attention_dropout, training=True)
        ctx = torch.bmm(probs.view(b * self.nh, s, s), vh)          # [b*nh, s, d]
        return ctx.view(b, self.nh, s, self.hd).permute(2, 0, 1, 3).reshape(s, b, self.nh * self.hd)

    def core_attention_context_parallel(self, qkv, training):
        """Context parallelism: ``qkv`` holds this CP rank's contiguous
        sequence chunk; two all-to-alls re-shard it to the FULL sequence for nh/cp heads around the
        unchanged causal flash kernel (parallel/context_parallel.py) and back."""
        from ..parallel.context_parallel import ulysses_attention
        st = ps.get_state()
        q, k, v = SF._qkv_views(qkv, self.nh, self.nkv, self.hd, False)   # [s/cp, b, heads, d]
        p = self.cfg.attention_dropout if training else 0.0
        if not self.cfg.use_flash_attn:
            raise NotImplementedError("context parallelism runs attention through the flash kernels "
                                      "(--use-flash-attn)")
        ctx = ulysses_attention(q, k, v, group=st.cp_group, causal=True, scale=1.0 / math.sqrt(self.hd),
                                dropout_p=p, rng=get_rng("tp"))
        return ctx.reshape(ctx.shape[0], ctx.shape[1], self.nh * self.hd)

    def forward(self, x, training=True):
        qkv = self.qkv(x)                                        # [s, b, (nh + 2 nkv) d]
        if _PACK["idx"] is not None:                              # padding-free micro-batch
            if self._groups_ok(qkv):
                return self.proj(self._attend_groups(qkv, training))
            return self.proj(_pack_rows(self._attend(_unpack_rows(qkv), training)))
        return self.proj(self._attend(qkv, training))            # (out, bias)

    def _groups_ok(self, qkv) -> bool:
        g = _PACK.get("groups")
        W = qkv.shape[-1]
        return (g is not None and self.cfg.use_flash_attn and ps.get_state().cp == 1 and _ext.use_kernels(qkv)
                and self.hd in (64, 128) and qkv.dtype in (torch.bfloat16, torch.float16)
                and (W * qkv.element_size()) % 16 == 0 and W % 8 == 0)

    def _attend_groups(self, qkv, training):
        """Padding-free attention in the length-grouped layout (``length_groups``): [T, 1, W]
        packed QKV -> grouped blocks (one row gather) -> RoPE -> causal flash per block -> [T, 1,
        nh hd] (one row gather)."""
        g = _PACK["groups"]
        W = qkv.shape[-1]
        x = _GatherRows.apply(qkv.reshape(-1, W), g["inv"], g["pack"])           # [P, W]
        if self.rope is not None:
            cos, sin, rot = self.rope
            x = _RopeQKVGroups.apply(x, cos, sin, rot, self.nh, self.nkv, self.hd, g["blocks"])
        p = self.cfg.attention_dropout if training else 0.0
        seeds = [SF._rng(get_rng("tp")).next() if p > 0 else (0, 0) for _ in g["blocks"]]
        ctx = _FlashQKVGroups.apply(x, self.nh, self.nkv, self.hd, 1.0 / math.sqrt(self.hd), float(p), seeds,
                                    g["blocks"])
        return _GatherRows.apply(ctx, g["pack"], g["inv"]).unsqueeze(1)         # [T, 1, nh hd]

    def _attend(self, qkv, training):
        cp = ps.get_state().cp
        if self.rope is not None:
            cos, sin, rot = self.rope
            if cp > 1:  # this rank's positions: chunk cp_rank of the full sequence
                off = ps.get_state().cp_rank * qkv.shape[0]
                cos, sin = cos[off: off + qkv.shape[0]], sin[off: off + qkv.shape[0]]
            qkv = _RopeQKV.apply(qkv, cos, sin, rot, self.nh, self.nkv, self.hd)
        if cp > 1:
            return self.core_attention_context_parallel(qkv, training)
        if self.cfg.use_flash_attn:
            # attention dropout runs inside the flash kernels; heads are TP-sharded, so the mask
            # comes from the per-TP-rank stream (Megatron forks the model-parallel tracker here)
            p = self.cfg.attention_dropout if training else 0.0
            ctx = SF.flash_attention_qkv(qkv, self.nh, self.nkv, self.hd, seq_first=True, causal=True,
                                         dropout_p=p, rng=get_rng("tp"))
        elif training and self.cfg.recompute_granularity == "selective" and torch.is_grad_enabled():
            # Megatron's selective recompute: only the [b, np, s, s] scores / probabilities /
            # dropout of the unfused core attention are dropped and recomputed in backward (the
            # flash kernels never store them, so with flash there is nothing to recompute)
            ctx = rng_checkpoint(lambda t: self.core_attention_unfused(t, training), qkv)
        else:
            ctx = self.core_attention_unfused(qkv, training)
        return ctx


class _RopeQKV(torch.autograd.Function):
    """RoPE on the q and k parts of a fused [s, b, W] QKV buffer (kernel: rope.hip), in place:
    the buffer is the QKV GEMM's own output (or the padding-free scatter's), which nothing else
    keeps, and its gradient comes straight from the attention backward — so neither direction
    pays a [tokens, W] copy (LLaMA-7B: 2 x 32 copies of 100-300 MB per step)."""

    @staticmethod
    def forward(ctx, qkv, cos, sin, rot, nh, nkv, hd):
        s, b, W = qkv.shape
        # a view (e.g. the [s, b, W] reshape of a TP linear's output under CP) cannot be marked
        # dirty inside a custom Function, so it takes the copy
        if qkv.is_contiguous() and qkv._base is None:
            out = qkv
            ctx.mark_dirty(qkv)
        else:
            out = qkv.contiguous()
        _apply_rope_parts(out.view(s * b, W), cos, sin, rot, nh, nkv, hd, b, s, False)
        ctx.save_for_backward(cos, sin)
        ctx.cfg = (rot, nh, nkv, hd, b, s)
        return out

    @staticmethod
    def backward(ctx, g):
        cos, sin = ctx.saved_tensors
        rot, nh, nkv, hd, b, s = ctx.cfg
        d = g if g.is_contiguous() else g.contiguous()
        _apply_rope_parts(d.view(s * b, -1), cos, sin, rot, nh, nkv, hd, b, s, True)
        return d, None, None, None, None, None, None


def _apply_rope_parts(flat, cos, sin, rot, nh, nkv, hd, b, s, inverse):
    q = flat[:, : nh * hd].view(s * b, nh, hd)
    k = flat[:, nh * hd:(nh + nkv) * hd].view(s * b, nkv, hd)
    from ..ops import _ext
    if _ext.use_kernels(flat):
        # q and k heads are adjacent in every row of the fused buffer and rotate identically:
        # ONE launch over the [tokens, nh + nkv, hd] view (row stride W)
        _ext.ext().rope_(flat[:, :(nh + nkv) * hd].view(s * b, nh + nkv, hd), cos, sin, rot, b, s, inverse)
    else:
        pos = torch.arange(s * b, device=flat.device) // b
        q.copy_(SF._rope_ref(q, cos.to(flat.device), sin.to(flat.device), rot, pos, inverse))
        k.copy_(SF._rope_ref(k, cos.to(flat.device), sin.to(flat.device), rot, pos, inverse))


class ParallelMLP(nn.Module):
    def __init__(self, cfg: TransformerConfig, layer_number: int, device=None, key: Optional[str] = None):
        super().__init__()
        self.cfg = cfg
        key = key or f"layers.{layer_number}"
        f = cfg.ffn_hidden_size
        std = cfg.init_method_std
        out_std = std / math.sqrt(2.0 * cfg.num_layers)
        self.gated = cfg.activation == "swiglu"
        fc1_out = 2 * f if self.gated else f
        self.fc1 = tp.ColumnParallelLinear(cfg.hidden_size, fc1_out, bias=cfg.add_bias_linear, init_std=std,
                                           key=f"{key}.fc1", seed=cfg.seed,
                                           params_dtype=cfg.params_dtype, device=device,
                                           sequence_parallel=cfg.sequence_parallel, skip_bias_add=True,
                                           chunks=[f, f] if self.gated else None,
                                           async_tensor_model_parallel_allreduce=cfg.async_tensor_model_parallel_allreduce,
                                           bias_grad_from_output=True)   # forward() only ever uses h + b
        self.fc2 = tp.RowParallelLinear(f, cfg.hidden_size, bias=cfg.add_bias_linear, init_std=out_std,
                                        key=f"{key}.fc2", seed=cfg.seed,
                                        params_dtype=cfg.params_dtype, device=device,
                                        sequence_parallel=cfg.sequence_parallel, skip_bias_add=True)

    def forward(self, x):
        act = self.cfg.activation
        if act == "gelu" and self.cfg.bias_gelu_fusion:
            # the fused forms read fc1 / fc2 weights without calling fc1(x) / fc2(x)
            _gather_wait(self.fc1, x)
            _gather_wait(self.fc2, x)
        if act == "gelu" and self.cfg.bias_gelu_fusion and tp.sp_fused_gelu_mlp_ok(x, self):
            # TP > 1 + sequence parallelism: the GeLU halves inside the ring-chunk GEMMs
            return tp.SPFusedGeLUMLP.apply(x, self.fc1.weight, self.fc1.bias, self.fc2.weight), self.fc2.bias
        if act == "gelu" and self.cfg.bias_gelu_fusion and tp.linear_bias_gelu_ok(x, self.fc1):
            if tp.fused_gelu_mlp_ok(x, self):
                # both GeLU halves inside the GEMMs: fc1 + bias + GeLU forward, fc2 dgrad + GeLU
                # backward (gemm_tn.hip epilogues)
                y = tp.FusedGeLUMLP.apply(x, self.fc1.weight, self.fc1.bias, self.fc2.weight)
                return y, self.fc2.bias
            # fc1 GEMM + bias + GeLU in one launch (gemm_tn.hip's bias-GeLU epilogue)
            return self.fc2(tp.linear_bias_gelu(x, self.fc1))
        h, b = self.fc1(x)
        if act in ("gelu", "gelu_erf"):
            if self.cfg.bias_gelu_fusion:
                h = SF.bias_gelu(h, b, "tanh" if act == "gelu" else "none")
            else:
                h = F.gelu(h + b if b is not None else h, approximate="tanh" if act == "gelu" else "none")
        elif act == "swiglu":
            if b is not None:
                h = h + b
            h = SF.swiglu(h)
        elif act == "squared_relu":
            h = F.relu(h + b if b is not None else h).pow(2)
        elif act == "relu":  # OPT
            h = F.relu(h + b if b is not None else h)
        else:
            raise ValueError(f"unknown activation {act}")
        return self.fc2(h)


class SwitchMLP(nn.Module):
    """``--num-experts E``: Megatron's Switch MLP (top-1 routing; the flag at
    /root/reference/3_training_megatron-lm/megatron/arguments.py:610-611, no expert-parallel group
    there either). A router (h -> E, softmax in fp32) picks one expert per token; each expert is a
    full ``ParallelMLP`` (tensor-parallel like the dense MLP); the token's output is the expert's
    (output + bias) scaled by the router probability. Tokens are sorted by expert once, so each
    expert runs ONE contiguous GEMM chain on its slice (no per-expert masks or scatters), and one
    gather puts the rows back. The per-expert token counts are read on the host (one sync per layer),
    so an MoE step is not graph-captured."""

    def __init__(self, cfg: TransformerConfig, layer_number: int, device=None):
        super().__init__()
        if cfg.sequence_parallel and ps.get_state().tp > 1:
            # each TP rank would route a different sequence shard, so the experts' TP collectives
            # would not line up across the group
            raise NotImplementedError("--num-experts with --sequence-parallel")
        self.cfg = cfg
        e = int(cfg.num_experts)
        self.router = nn.Parameter(tp.init_full_then_shard(
            (e, cfg.hidden_size), cfg.init_method_std, f"layers.{layer_number}.router", cfg.seed,
            cfg.params_dtype, device, None, 0, 1))
        self.router_bias = nn.Parameter(torch.zeros(e, dtype=cfg.params_dtype, device=device))
        self.experts = nn.ModuleList(ParallelMLP(cfg, layer_number, device, key=f"layers.{layer_number}.experts.{i}")
                                     for i in range(e))

    def route(self, flat):
        """(top-1 probability [n] fp32, expert index [n]) of each token row."""
        prob = torch.softmax(F.linear(flat, self.router, self.router_bias).float(), dim=-1)
        return prob.max(dim=-1)

    def forward(self, x):
        s, b, h = x.shape
        flat = x.reshape(s * b, h)
        top_p, top_e = self.route(flat)
        order = torch.argsort(top_e, stable=True)
        counts = torch.bincount(top_e, minlength=len(self.experts)).tolist()
        xs = flat.index_select(0, order)
        outs, o = [], 0
        for i, n in enumerate(counts):
            if n == 0:
                continue          # an expert with no tokens gets no gradient this step
            y, yb = self.experts[i](xs[o:o + n].unsqueeze(1))
            y = y.squeeze(1)
            outs.append(y + yb if yb is not None else y)
            o += n
        inv = torch.empty_like(order)
        inv[order] = torch.arange(order.numel(), device=order.device)
        out = torch.cat(outs).index_select(0, inv) * top_p.unsqueeze(-1).to(x.dtype)
        return out.view(s, b, h), None


def _sp_gather(cfg):
    """(tp, tp_rank) when sequence-parallel norms should write into all-gather slots."""
    if not cfg.sequence_parallel or _PACK["idx"] is not None:
        return None
    return tp.sp_gather_spec()


class ParallelTransformerLayer(nn.Module):
    def __init__(self, cfg: TransformerConfig, layer_number: int, device=None):
        super().__init__()
        self.cfg = cfg
        self.layer_number = layer_number
        self.input_norm = Norm(cfg.hidden_size, cfg, device)
        self.attention = ParallelAttention(cfg, layer_number, device)
        self.post_attention_norm = Norm(cfg.hidden_size, cfg, device)
        self.mlp = SwitchMLP(cfg, layer_number, device) if cfg.num_experts else ParallelMLP(cfg, layer_number, device)
        self.post_ln_residual = bool(cfg.apply_residual_connection_post_layernorm)
        if self.post_ln_residual and cfg.sequence_parallel and ps.get_state().tp > 1:
            # the SP norms hand their output to the all-gather, not back as a local residual
            raise NotImplementedError("--apply-residual-connection-post-layernorm with --sequence-parallel")

    def forward(self, x, xbias, residual):
        training = self.training
        p = self.cfg.hidden_dropout
        # sequence parallelism: each norm's output is all-gathered by the next column-parallel
        # linear and (after a layer) its input gradient by the row-parallel linear that produced
        # x — both are written straight into their slot of the gather buffer (no local copy)
        g = _sp_gather(self.cfg)
        ln1, residual = self.input_norm.fused(x, xbias, residual, p, training,
                                              gather=None if g is None else g + (True, residual is not None))
        if self.post_ln_residual:           # Megatron's --apply-residual-connection-post-layernorm
            residual = ln1
        a, ab = self.attention(ln1, training)
        ln2, residual = self.post_attention_norm.fused(a, ab, residual, p, training,
                                                       gather=None if g is None else g + (True, True))
        if self.post_ln_residual:
            residual = ln2
        m, mb = self.mlp(ln2)
        return m, mb, residual

    def forward_phases(self, st):
        """``forward`` cut at its four sequence-parallel exchanges for the sub-batch interleave
        (``ParallelTransformer._forward_subbatch``): each phase ends right after it STARTS an
        exchange (the norms' all-gathers by ``tp.ag_start``; the row-parallel linears' reduce-
        scatters are left in flight by ``rs_ring`` under ``tp.begin_subbatch``) and the next phase
        of this half begins by completing it. ``st`` holds this half's (x, xbias, residual)."""
        training = self.training
        p = self.cfg.hidden_dropout
        g = _sp_gather(self.cfg)
        group = ps.get_state().tp_group
        x, residual = tp.rs_finish(st["x"]), st["residual"]
        ln1, residual = self.input_norm.fused(x, st["xbias"], residual, p, training,
                                              gather=None if g is None else g + (True, residual is not None))
        tp.ag_start(ln1, group)
        yield
        a, ab = self.attention(ln1, training)
        yield
        ln2, residual = self.post_attention_norm.fused(tp.rs_finish(a), ab, residual, p, training,
                                                       gather=None if g is None else g + (True, True))
        tp.ag_start(ln2, group)
        yield
        m, mb = self.mlp(ln2)
        st.update(x=m, xbias=mb, residual=residual)
        yield


# Sub-batch interleave of the sequence-parallel TP-pair exchanges (tp.begin_subbatch). "2": the
# two batch halves of a micro-batch alternate phase by phase; "0" (default) off.
_SUBBATCH = int(os.environ.get("SMDT_SP_SUBBATCH", "0") or 0)


class ParallelTransformer(nn.Module):
    """A stack of layers [first, first + n) of the full model (pipeline stages own a slice)."""

    def __init__(self, cfg: TransformerConfig, first_layer: int, num_layers: int, post_norm: bool, device=None):
        super().__init__()
        self.cfg = cfg
        self.layers = nn.ModuleList([ParallelTransformerLayer(cfg, first_layer + i, device) for i in range(num_layers)])
        self.final_norm = Norm(cfg.hidden_size, cfg, device) if post_norm else None

    def _run(self, i, x, xb, res):
        layer = self.layers[i]
        cfg = self.cfg
        if self.training and cfg.recompute_granularity == "full":
            n = cfg.recompute_num_layers or len(self.layers)
            if cfg.recompute_method == "block" and i >= n:
                return layer(x, xb, res)
            if cfg.distribute_saved_activations and ps.get_state().tp > 1 and not cfg.sequence_parallel:
                from ..parallel.random import distributed_checkpoint
                if res is None:
                    return distributed_checkpoint(lambda a, b_: layer(a, b_, None), x, xb)
                return distributed_checkpoint(layer, x, xb, res)
            if xb is None:
                return rng_checkpoint(lambda a, r: layer(a, None, r), x, res)
            return rng_checkpoint(layer, x, xb, res)
        return layer(x, xb, res)

    def _subbatch_ok(self, x) -> bool:
        cfg = self.cfg
        st = ps.get_state()
        return (_SUBBATCH == 2 and self.training and torch.is_grad_enabled() and cfg.sequence_parallel
                and st.cp == 1 and cfg.recompute_granularity != "full" and _PACK["idx"] is None
                and tp.subbatch_capable(st) and x.dim() == 3 and x.shape[1] % 2 == 0
                and len(self.layers) > 0)

    def _forward_subbatch(self, x, xbias, residual):
        """The layer stack on the two batch halves of the micro-batch, phase by phase alternately
        (see ``ParallelTransformerLayer.forward_phases``): half b's GEMMs / attention run while half
        a's exchange is in flight and vice versa. The halves meet again (one concat each) before
        the final norm / the pipeline send. Same math as ``forward`` per half; with dropout, the
        masks are drawn in the interleaved order."""
        hb = x.shape[1] // 2
        if x.requires_grad:
            x = tp.WgradMergeScope.apply(x, False)
        halves = []
        for i in range(2):
            sl = slice(i * hb, (i + 1) * hb)
            halves.append({"x": x[:, sl].contiguous(), "xbias": xbias,
                           "residual": None if residual is None else residual[:, sl].contiguous()})
        tp.begin_subbatch()
        try:
            for layer in self.layers:
                gens = [layer.forward_phases(h) for h in halves]
                for _ in range(4):
                    for gen in gens:
                        next(gen)
            for h in halves:
                tp.rs_finish(h["x"])
        finally:
            tp.end_subbatch()
        x = torch.cat([h["x"] for h in halves], dim=1)
        if x.requires_grad:
            x = tp.WgradMergeScope.apply(x, True)
        xbias = halves[0]["xbias"]
        residual = torch.cat([h["residual"] for h in halves], dim=1)
        return x, xbias, residual

    def forward(self, x, xbias=None, residual=None):
        """Returns (pending_x, pending_bias, residual) or, with ``final_norm``, the normalised
        output (the pending branch folded into the residual first)."""
        if self._subbatch_ok(x):
            x, xbias, residual = self._forward_subbatch(x, xbias, residual)
        elif self.cfg.recompute_granularity != "full" and not tp.foreign_hooks(self):
            # every row-parallel output of the stack is consumed by the next fused norm (the
            # layers' own, or the final one): the ring reduce-scatters leave their combine to it.
            # Not with user hooks on the stack (they would read a tensor missing the peer's
            # partial); the ledger (tp.check_pending_adds) catches any other consumer.
            if x.requires_grad and torch.is_grad_enabled():
                x = tp.PendingAddCheck.apply(x)
            with tp.defer_rs_add():
                for i in range(len(self.layers)):
                    x, xbias, residual = self._run(i, x, xbias, residual)
        else:
            for i in range(len(self.layers)):
                x, xbias, residual = self._run(i, x, xbias, residual)
        if self.final_norm is not None:
            g = _sp_gather(self.cfg)          # y feeds the LM head's column-parallel all-gather
            y, _ = self.final_norm.fused(x, xbias, residual, self.cfg.hidden_dropout, self.training,
                                         gather=None if g is None else g + (True, residual is not None))
            tp.check_pending_adds("the end of the layer stack's forward")
            return y
        x = tp.materialize_add(x)      # leaves the stage: no pending summand
        tp.check_pending_adds("the end of the layer stack's forward")
        return x, xbias, residual
