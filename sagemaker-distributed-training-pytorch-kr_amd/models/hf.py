"""HuggingFace-compatible causal LMs (OPT, LLaMA, GPT-2) on the MI355X transformer stack.

The Alpaca recipe calls ``transformers.AutoModelForCausalLM.from_pretrained(model_name_or_path)``
(/root/reference/4_training_alpaca_deepspeed/train.py:214-217; NB4 runs facebook/opt-125m, the
BASELINE config names LLaMA-7B). Here the same architectures are expressed as
``smdt_amd.models.gpt.GPTModel`` (fused BDA+norm, flash attention, fused CE, SwiGLU, RoPE HIP
kernels) and HF checkpoints are converted on load / save:

  * ``config_from_hf(dict)``       HF ``config.json`` -> TransformerConfig
  * ``HFCausalLM.from_pretrained`` local dir with config.json + *.safetensors / pytorch_model.bin
                                   (``weights_only``), or a built-in config name (random init —
                                   there is no network to download weights)
  * ``save_pretrained(dir)``       writes HF names + config.json (+ safetensors) so the result
                                   loads back in ``transformers``
  * ``forward(input_ids, attention_mask, labels)`` HF semantics: labels are shifted inside and
                                   ``-100`` is ignored; returns ``(loss, None)``.
"""
from __future__ import annotations

import json
import os
from typing import Dict, Optional

import torch
import torch.nn as nn

from .gpt import GPTModel
from .transformer import TransformerConfig

BUILTIN = {
    "facebook/opt-125m": {"model_type": "opt", "hidden_size": 768, "num_hidden_layers": 12, "num_attention_heads": 12,
                          "ffn_dim": 3072, "vocab_size": 50272, "max_position_embeddings": 2048,
                          "activation_function": "relu", "do_layer_norm_before": True, "enable_bias": True,
                          "word_embed_proj_dim": 768, "pad_token_id": 1, "bos_token_id": 2, "eos_token_id": 2},
    "facebook/opt-1.3b": {"model_type": "opt", "hidden_size": 2048, "num_hidden_layers": 24, "num_attention_heads": 32,
                          "ffn_dim": 8192, "vocab_size": 50272, "max_position_embeddings": 2048,
                          "activation_function": "relu", "do_layer_norm_before": True, "enable_bias": True,
                          "word_embed_proj_dim": 2048, "pad_token_id": 1, "bos_token_id": 2, "eos_token_id": 2},
    "llama-7b": {"model_type": "llama", "hidden_size": 4096, "num_hidden_layers": 32, "num_attention_heads": 32,
                 "num_key_value_heads": 32, "intermediate_size": 11008, "vocab_size": 32000,
                 "max_position_embeddings": 2048, "rms_norm_eps": 1e-6, "rope_theta": 10000.0, "hidden_act": "silu",
                 "tie_word_embeddings": False, "bos_token_id": 1, "eos_token_id": 2},
    "gpt2": {"model_type": "gpt2", "n_embd": 768, "n_layer": 12, "n_head": 12, "vocab_size": 50257, "n_positions": 1024,
             "layer_norm_epsilon": 1e-5, "activation_function": "gelu_new"},
}
BUILTIN["huggyllama/llama-7b"] = BUILTIN["llama-7b"]
BUILTIN["meta-llama/Llama-2-7b-hf"] = dict(BUILTIN["llama-7b"], max_position_embeddings=4096)


def _round_up(x, m):
    return ((x + m - 1) // m) * m


def config_from_hf(hf: Dict, params_dtype=torch.bfloat16, vocab_multiple: int = 128, **over) -> TransformerConfig:
    mt = hf.get("model_type", "llama")
    if mt == "opt":
        assert hf.get("word_embed_proj_dim", hf["hidden_size"]) == hf["hidden_size"], \
            "OPT variants with project_in/out (opt-350m) are not supported"
        assert hf.get("do_layer_norm_before", True), "post-LN OPT variants are not supported"
        cfg = dict(num_layers=hf["num_hidden_layers"], hidden_size=hf["hidden_size"],
                   num_attention_heads=hf["num_attention_heads"], ffn_hidden_size=hf["ffn_dim"],
                   activation="relu" if hf.get("activation_function", "relu") == "relu" else "gelu_erf",
                   normalization="LayerNorm", add_bias_linear=hf.get("enable_bias", True),
                   position_embedding_type="learned_absolute", max_position_embeddings=hf["max_position_embeddings"],
                   position_offset=2, layernorm_epsilon=1e-5, untie_embeddings_and_output_weights=False)
    elif mt in ("llama", "mistral"):
        cfg = dict(num_layers=hf["num_hidden_layers"], hidden_size=hf["hidden_size"],
                   num_attention_heads=hf["num_attention_heads"],
                   num_query_groups=hf.get("num_key_value_heads", hf["num_attention_heads"]),
                   ffn_hidden_size=hf["intermediate_size"], activation="swiglu", normalization="RMSNorm",
                   add_bias_linear=False, position_embedding_type="rope",
                   rotary_base=hf.get("rope_theta", 10000.0), max_position_embeddings=hf["max_position_embeddings"],
                   layernorm_epsilon=hf.get("rms_norm_eps", 1e-6),
                   untie_embeddings_and_output_weights=not hf.get("tie_word_embeddings", False))
    elif mt == "gpt2":
        cfg = dict(num_layers=hf["n_layer"], hidden_size=hf["n_embd"], num_attention_heads=hf["n_head"],
                   ffn_hidden_size=4 * hf["n_embd"], activation="gelu", normalization="LayerNorm",
                   add_bias_linear=True, position_embedding_type="learned_absolute",
                   max_position_embeddings=hf["n_positions"], layernorm_epsilon=hf.get("layer_norm_epsilon", 1e-5),
                   untie_embeddings_and_output_weights=False)
    else:
        raise ValueError(f"unsupported model_type {mt}")
    cfg.update(padded_vocab_size=_round_up(hf["vocab_size"], vocab_multiple), hidden_dropout=0.0,
               attention_dropout=0.0, params_dtype=params_dtype)
    cfg.update(over)
    return TransformerConfig(**cfg)


# ----------------------------------------------------------------------------------- name maps

def _hf_to_ours(hf: Dict, sd: Dict[str, torch.Tensor], ncfg: TransformerConfig) -> Dict[str, torch.Tensor]:
    mt = hf.get("model_type")
    out = {}
    L = ncfg.num_layers
    if mt == "opt":
        p = "model.decoder."
        if p + "embed_tokens.weight" not in sd and "decoder.embed_tokens.weight" in sd:
            p = "decoder."
        out["embedding.weight"] = sd[p + "embed_tokens.weight"]
        out["position_embeddings"] = sd[p + "embed_positions.weight"]
        for i in range(L):
            a = f"{p}layers.{i}."
            o = f"decoder.layers.{i}."
            out[o + "attention.qkv.weight"] = torch.cat([sd[a + f"self_attn.{x}_proj.weight"] for x in "qkv"], 0)
            out[o + "attention.qkv.bias"] = torch.cat([sd[a + f"self_attn.{x}_proj.bias"] for x in "qkv"], 0)
            out[o + "attention.proj.weight"] = sd[a + "self_attn.out_proj.weight"]
            out[o + "attention.proj.bias"] = sd[a + "self_attn.out_proj.bias"]
            out[o + "input_norm.weight"] = sd[a + "self_attn_layer_norm.weight"]
            out[o + "input_norm.bias"] = sd[a + "self_attn_layer_norm.bias"]
            out[o + "post_attention_norm.weight"] = sd[a + "final_layer_norm.weight"]
            out[o + "post_attention_norm.bias"] = sd[a + "final_layer_norm.bias"]
            out[o + "mlp.fc1.weight"] = sd[a + "fc1.weight"]
            out[o + "mlp.fc1.bias"] = sd[a + "fc1.bias"]
            out[o + "mlp.fc2.weight"] = sd[a + "fc2.weight"]
            out[o + "mlp.fc2.bias"] = sd[a + "fc2.bias"]
        out["decoder.final_norm.weight"] = sd[p + "final_layer_norm.weight"]
        out["decoder.final_norm.bias"] = sd[p + "final_layer_norm.bias"]
    elif mt in ("llama", "mistral"):
        out["embedding.weight"] = sd["model.embed_tokens.weight"]
        for i in range(L):
            a = f"model.layers.{i}."
            o = f"decoder.layers.{i}."
            out[o + "attention.qkv.weight"] = torch.cat([sd[a + f"self_attn.{x}_proj.weight"] for x in "qkv"], 0)
            out[o + "attention.proj.weight"] = sd[a + "self_attn.o_proj.weight"]
            out[o + "mlp.fc1.weight"] = torch.cat([sd[a + "mlp.gate_proj.weight"], sd[a + "mlp.up_proj.weight"]], 0)
            out[o + "mlp.fc2.weight"] = sd[a + "mlp.down_proj.weight"]
            out[o + "input_norm.weight"] = sd[a + "input_layernorm.weight"]
            out[o + "post_attention_norm.weight"] = sd[a + "post_attention_layernorm.weight"]
        out["decoder.final_norm.weight"] = sd["model.norm.weight"]
        if "lm_head.weight" in sd:
            out["output_weight"] = sd["lm_head.weight"]
    elif mt == "gpt2":
        pre = "transformer." if "transformer.wte.weight" in sd else ""
        out["embedding.weight"] = sd[pre + "wte.weight"]
        out["position_embeddings"] = sd[pre + "wpe.weight"]
        for i in range(L):
            a = f"{pre}h.{i}."
            o = f"decoder.layers.{i}."
            out[o + "attention.qkv.weight"] = sd[a + "attn.c_attn.weight"].t()
            out[o + "attention.qkv.bias"] = sd[a + "attn.c_attn.bias"]
            out[o + "attention.proj.weight"] = sd[a + "attn.c_proj.weight"].t()
            out[o + "attention.proj.bias"] = sd[a + "attn.c_proj.bias"]
            out[o + "input_norm.weight"] = sd[a + "ln_1.weight"]
            out[o + "input_norm.bias"] = sd[a + "ln_1.bias"]
            out[o + "post_attention_norm.weight"] = sd[a + "ln_2.weight"]
            out[o + "post_attention_norm.bias"] = sd[a + "ln_2.bias"]
            out[o + "mlp.fc1.weight"] = sd[a + "mlp.c_fc.weight"].t()
            out[o + "mlp.fc1.bias"] = sd[a + "mlp.c_fc.bias"]
            out[o + "mlp.fc2.weight"] = sd[a + "mlp.c_proj.weight"].t()
            out[o + "mlp.fc2.bias"] = sd[a + "mlp.c_proj.bias"]
        out["decoder.final_norm.weight"] = sd[pre + "ln_f.weight"]
        out["decoder.final_norm.bias"] = sd[pre + "ln_f.bias"]
    return out


def _ours_to_hf(hf: Dict, sd: Dict[str, torch.Tensor], ncfg: TransformerConfig, vocab: int) -> Dict[str, torch.Tensor]:
    mt = hf.get("model_type")
    out = {}
    L = ncfg.num_layers
    h = ncfg.num_attention_heads * ncfg.kv_channels
    kv = ncfg.num_query_groups * ncfg.kv_channels
    emb = sd["embedding.weight"][:vocab]
    if mt == "opt":
        p = "model.decoder."
        out[p + "embed_tokens.weight"] = emb
        out[p + "embed_positions.weight"] = sd["position_embeddings"]
        for i in range(L):
            a, o = f"{p}layers.{i}.", f"decoder.layers.{i}."
            q, k, v = torch.split(sd[o + "attention.qkv.weight"], [h, kv, kv], 0)
            qb, kb, vb = torch.split(sd[o + "attention.qkv.bias"], [h, kv, kv], 0)
            for n, w, b in (("q", q, qb), ("k", k, kb), ("v", v, vb)):
                out[a + f"self_attn.{n}_proj.weight"], out[a + f"self_attn.{n}_proj.bias"] = w, b
            out[a + "self_attn.out_proj.weight"] = sd[o + "attention.proj.weight"]
            out[a + "self_attn.out_proj.bias"] = sd[o + "attention.proj.bias"]
            out[a + "self_attn_layer_norm.weight"] = sd[o + "input_norm.weight"]
            out[a + "self_attn_layer_norm.bias"] = sd[o + "input_norm.bias"]
            out[a + "final_layer_norm.weight"] = sd[o + "post_attention_norm.weight"]
            out[a + "final_layer_norm.bias"] = sd[o + "post_attention_norm.bias"]
            for n in ("fc1", "fc2"):
                out[a + f"{n}.weight"] = sd[o + f"mlp.{n}.weight"]
                out[a + f"{n}.bias"] = sd[o + f"mlp.{n}.bias"]
        out[p + "final_layer_norm.weight"] = sd["decoder.final_norm.weight"]
        out[p + "final_layer_norm.bias"] = sd["decoder.final_norm.bias"]
        out["lm_head.weight"] = emb
    elif mt in ("llama", "mistral"):
        out["model.embed_tokens.weight"] = emb
        f = ncfg.ffn_hidden_size
        for i in range(L):
            a, o = f"model.layers.{i}.", f"decoder.layers.{i}."
            q, k, v = torch.split(sd[o + "attention.qkv.weight"], [h, kv, kv], 0)
            out[a + "self_attn.q_proj.weight"], out[a + "self_attn.k_proj.weight"], out[a + "self_attn.v_proj.weight"] = q, k, v
            out[a + "self_attn.o_proj.weight"] = sd[o + "attention.proj.weight"]
            g, u = torch.split(sd[o + "mlp.fc1.weight"], [f, f], 0)
            out[a + "mlp.gate_proj.weight"], out[a + "mlp.up_proj.weight"] = g, u
            out[a + "mlp.down_proj.weight"] = sd[o + "mlp.fc2.weight"]
            out[a + "input_layernorm.weight"] = sd[o + "input_norm.weight"]
            out[a + "post_attention_layernorm.weight"] = sd[o + "post_attention_norm.weight"]
        out["model.norm.weight"] = sd["decoder.final_norm.weight"]
        out["lm_head.weight"] = sd["output_weight"][:vocab] if "output_weight" in sd else emb
    elif mt == "gpt2":
        out["transformer.wte.weight"] = emb
        out["transformer.wpe.weight"] = sd["position_embeddings"]
        for i in range(L):
            a, o = f"transformer.h.{i}.", f"decoder.layers.{i}."
            out[a + "attn.c_attn.weight"] = sd[o + "attention.qkv.weight"].t()
            out[a + "attn.c_attn.bias"] = sd[o + "attention.qkv.bias"]
            out[a + "attn.c_proj.weight"] = sd[o + "attention.proj.weight"].t()
            out[a + "attn.c_proj.bias"] = sd[o + "attention.proj.bias"]
            out[a + "ln_1.weight"], out[a + "ln_1.bias"] = sd[o + "input_norm.weight"], sd[o + "input_norm.bias"]
            out[a + "ln_2.weight"], out[a + "ln_2.bias"] = sd[o + "post_attention_norm.weight"], sd[o + "post_attention_norm.bias"]
            out[a + "mlp.c_fc.weight"] = sd[o + "mlp.fc1.weight"].t()
            out[a + "mlp.c_fc.bias"] = sd[o + "mlp.fc1.bias"]
            out[a + "mlp.c_proj.weight"] = sd[o + "mlp.fc2.weight"].t()
            out[a + "mlp.c_proj.bias"] = sd[o + "mlp.fc2.bias"]
        out["transformer.ln_f.weight"] = sd["decoder.final_norm.weight"]
        out["transformer.ln_f.bias"] = sd["decoder.final_norm.bias"]
        out["lm_head.weight"] = emb
    return {k: v.contiguous() for k, v in out.items()}


def _load_state_dict_files(path: str) -> Dict[str, torch.Tensor]:
    sd = {}
    files = sorted(os.listdir(path))
    st = [f for f in files if f.endswith(".safetensors")]
    if st:
        from safetensors.torch import load_file
        for f in st:
            sd.update(load_file(os.path.join(path, f)))
        return sd
    bins = [f for f in files if f.startswith("pytorch_model") and f.endswith(".bin")]
    for f in bins:
        sd.update(torch.load(os.path.join(path, f), map_location="cpu", weights_only=True))
    if not sd:
        raise FileNotFoundError(f"no *.safetensors / pytorch_model*.bin under {path}")
    return sd


class HFCausalLM(nn.Module):
    """HF-style causal LM facade over ``GPTModel``."""

    def __init__(self, hf_config: Dict, params_dtype=torch.bfloat16, device=None, **over):
        super().__init__()
        self.hf_config = dict(hf_config)
        self.vocab_size = int(hf_config["vocab_size"])
        self.cfg = config_from_hf(self.hf_config, params_dtype, **over)
        self.model = GPTModel(self.cfg, device=device)
        self.model.loss_vocab_size = self.vocab_size
        self.config = _AttrDict(self.hf_config)

    # ---- construction
    @classmethod
    def from_pretrained(cls, name_or_path: str, params_dtype=torch.bfloat16, device=None, cache_dir=None, **over):
        path = name_or_path
        if cache_dir and not os.path.isdir(path):
            cand = os.path.join(cache_dir, name_or_path)
            path = cand if os.path.isdir(cand) else path
        if os.path.isdir(path) and os.path.exists(os.path.join(path, "config.json")):
            hf = json.load(open(os.path.join(path, "config.json")))
            m = cls(hf, params_dtype, device, **over)
            try:
                sd = _load_state_dict_files(path)
            except FileNotFoundError:
                print(f"[smdt] {path}: config only, random init", flush=True)
                return m
            ours = _hf_to_ours(hf, sd, m.cfg)
            m.load_our_state_dict(ours)
            return m
        if name_or_path in BUILTIN:
            print(f"[smdt] '{name_or_path}': weights are not available offline; building the architecture "
                  "with random init", flush=True)
            return cls(BUILTIN[name_or_path], params_dtype, device, **over)
        raise FileNotFoundError(f"{name_or_path}: not a local HF model dir and not a built-in config")

    @torch.no_grad()
    def load_our_state_dict(self, ours: Dict[str, torch.Tensor]):
        """Copy a state dict in; parameters partitioned by parallel/zero_init.Init keep only their
        shard of each tensor (no gather)."""
        from ..parallel import zero_init as zi
        own = dict(self.model.named_parameters())
        for k, v in ours.items():
            if k not in own:
                continue
            p = own[k]
            shape = zi.logical_shape(p)
            if shape != tuple(v.shape):
                if k in ("embedding.weight", "output_weight") and v.shape[0] <= shape[0]:
                    full = torch.zeros(shape, dtype=p.dtype)
                    full[: v.shape[0]].copy_(v.to(p.dtype))
                    v = full
                else:
                    raise ValueError(f"shape mismatch for {k}: {tuple(v.shape)} vs {shape}")
            zi.load_full_(p, v.to(p.device))

    def save_pretrained(self, out_dir: str, state_dict: Optional[Dict[str, torch.Tensor]] = None,
                        safe_serialization: bool = True):
        os.makedirs(out_dir, exist_ok=True)
        sd = state_dict or {k: v.detach().cpu() for k, v in self.model.state_dict().items()}
        hf_sd = _ours_to_hf(self.hf_config, sd, self.cfg, self.vocab_size)
        cfg = dict(self.hf_config)
        cfg["vocab_size"] = self.vocab_size
        cfg.setdefault("torch_dtype", str(self.cfg.params_dtype).replace("torch.", ""))
        arch = {"opt": "OPTForCausalLM", "llama": "LlamaForCausalLM", "mistral": "MistralForCausalLM",
                "gpt2": "GPT2LMHeadModel"}.get(cfg.get("model_type"), "")
        cfg.setdefault("architectures", [arch])
        with open(os.path.join(out_dir, "config.json"), "w") as f:
            json.dump(cfg, f, indent=2)
        if safe_serialization:
            from safetensors.torch import save_file
            if cfg.get("model_type") in ("opt", "gpt2") or not self.cfg.untie_embeddings_and_output_weights:
                hf_sd.pop("lm_head.weight", None)  # tied
            save_file({k: v.contiguous() for k, v in hf_sd.items()}, os.path.join(out_dir, "model.safetensors"),
                      metadata={"format": "pt"})
        else:
            torch.save(hf_sd, os.path.join(out_dir, "pytorch_model.bin"))

    # ---- HF helpers used by smart_tokenizer_and_embedding_resize
    def resize_token_embeddings(self, new_num_tokens: int):
        """Grow the (padded) vocab; rows beyond the old vocab are zero until the caller fills them.

        The embedding / LM-head Parameter objects are kept and only their data grows, so a model
        built under parallel/zero_init.Init — resized inside ``zero_init.gathered([...])``, as the
        recipe does (train.py) — has the GROWN tensors cut back into shards when that block exits
        (new Parameter objects would have stayed full on every rank while the old ones were
        re-cut), and DDP flags such as the tied embedding's two gradient contributions stay."""
        self.vocab_size = int(new_num_tokens)
        self.hf_config["vocab_size"] = self.vocab_size
        self.model.loss_vocab_size = self.vocab_size
        need = _round_up(new_num_tokens, 128)
        if need <= self.cfg.padded_vocab_size:
            return self
        from ..parallel import zero_init as zi

        def grow(p):
            if zi.is_partitioned(p):
                raise RuntimeError("resize_token_embeddings on a partitioned parameter: call it inside "
                                   "zero_init.gathered([...]) (recipes/4_training_alpaca_deepspeed/train.py)")
            neww = torch.zeros(need, p.shape[1], dtype=p.dtype, device=p.device)
            neww[: p.shape[0]] = p.data
            p.data = neww
        self.cfg.padded_vocab_size = need
        with torch.no_grad():
            emb = self.model.embedding
            grow(emb.weight)
            emb.num_embeddings = emb.per = need
            emb.vocab_end = need
            if self.model.output_weight is not None:
                grow(self.model.output_weight)
            if not self.cfg.untie_embeddings_and_output_weights:
                self.model.embedding.weight._smdt_grad_contributions = 2
        return self

    def get_input_embeddings(self):
        return self.model.embedding

    def get_output_embeddings(self):
        class _W:  # exposes .weight like an nn.Linear head
            pass
        w = _W()
        w.weight = self.model.output_weight if self.model.output_weight is not None else self.model.embedding.weight
        return w

    # ---- forward
    def _pack_index(self, attention_mask):
        """Seq-first flat indices of the real tokens when the micro-batch can run padding-free
        (models/transformer.py ``packed_sequences``): a right-padded CPU mask (no device sync),
        no tensor / pipeline / context parallelism, and some padding to save. Else None."""
        if (attention_mask is None or os.environ.get("SMDT_SFT_UNPAD", "1") != "1"
                or attention_mask.device.type != "cpu" or attention_mask.dim() != 2):
            return None
        from ..parallel import state as ps
        st = ps.get_state() if ps.model_parallel_is_initialized() else None
        if st is not None and (st.tp > 1 or st.pp > 1 or st.cp > 1):
            return None
        m = attention_mask.bool()
        if bool(m.all()) or not bool(m[:, 0].all()) or bool((m[:, 1:] & ~m[:, :-1]).any()):
            return None                              # nothing to save, or not right-padded
        ms = m.t().reshape(-1)
        real = ms.nonzero().squeeze(1)
        # round the token count up to a multiple of 64 with pad positions (pads never reach a real
        # token under the causal mask and carry label -100): GEMM / wgrad tiles want M % 32 == 0
        need = -real.numel() % 64
        pads = (~ms).nonzero().squeeze(1)
        if pads.numel() < need or real.numel() + need >= ms.numel():
            return None
        return torch.cat([real, pads[:need]]).sort().values

    def forward(self, input_ids, attention_mask=None, labels=None, row_groups=None, **_):
        """Returns (mean loss over label tokens, per-token loss [b, s]) with HF shift semantics.
        With a right-padded CPU ``attention_mask`` the model runs on the real tokens only.
        ``row_groups`` (CPU long [b], optional): rows belong to micro-batches 0..G-1 of a fused
        accumulation window; the loss is then the mean over the groups of each group's own
        token-mean (exactly what G accumulated micro-batch backwards of loss / G produce)."""
        if labels is None:
            return None, self.model(input_ids)[..., : self.vocab_size]
        shifted = torch.full_like(labels, -100)
        shifted[:, :-1] = labels[:, 1:]
        idx = self._pack_index(attention_mask)
        if idx is not None:
            from . import transformer as _T
            from .transformer import packed_sequences
            b, L = input_ids.shape
            groups = (_T.length_groups(attention_mask.bool(), idx, input_ids.device,
                                       hidden=None if _T._LENGTH_GROUPS_FORCE else int(self.cfg.hidden_size))
                      if _T._LENGTH_GROUPS and input_ids.is_cuda else None)
            idx = idx.to(input_ids.device, non_blocking=True)
            tok = input_ids.t().reshape(-1).index_select(0, idx).unsqueeze(0)          # [1, T]
            pos = torch.div(idx, b, rounding_mode="floor").unsqueeze(0)                # position in its row
            lab = shifted.t().reshape(-1).index_select(0, idx).unsqueeze(0)
            self.last_computed_tokens = int(idx.numel())
            with packed_sequences(idx, b, L, groups):
                tl = self.model(tok, pos, None, labels=lab)                            # [1, T]
            valid = (lab != -100).float()
            rows = torch.remainder(idx, b) if row_groups is not None else None
            loss = _grouped_mean(tl.reshape(-1), valid.reshape(-1), rows, row_groups)
            tok_loss = tl.new_zeros(L * b).index_copy(0, idx, tl.reshape(-1)).view(L, b).t()
            return loss, tok_loss
        self.last_computed_tokens = int(input_ids.numel())
        tok_loss = self.model(input_ids, None, None, labels=shifted)
        valid = (shifted != -100).float()
        rows = (torch.arange(tok_loss.shape[0], device=tok_loss.device).unsqueeze(1).expand_as(tok_loss).reshape(-1)
                if row_groups is not None else None)
        loss = _grouped_mean(tok_loss.reshape(-1), valid.reshape(-1), rows, row_groups)
        return loss, tok_loss


def _grouped_mean(tl, valid, rows, row_groups):
    """Mean of per-group token-means (``row_groups[rows]`` = group of each token), or the plain
    token-mean without groups."""
    if row_groups is None:
        return (tl.float() * valid).sum() / valid.sum().clamp(min=1.0)
    grp = row_groups.to(tl.device, non_blocking=True).index_select(0, rows)
    G = int(row_groups.max()) + 1
    num = torch.zeros(G, device=tl.device, dtype=torch.float32).index_add_(0, grp, tl.float() * valid)
    den = torch.zeros(G, device=tl.device, dtype=torch.float32).index_add_(0, grp, valid)
    return (num / den.clamp(min=1.0)).mean()


class _AttrDict(dict):
    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e
