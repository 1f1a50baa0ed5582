"""HF-compatible causal LMs: weight conversion and loss parity against ``transformers``.

The Alpaca recipe loads ``AutoModelForCausalLM`` (reference 4_training_alpaca_deepspeed/train.py:214)
and saves HF checkpoints (train.py:245-246). These tests build tiny OPT / LLaMA(GQA) / GPT-2
models with our stack, save them in HF layout, load them with ``transformers`` and compare
losses/logits; then load back and check the round trip.
"""
import tempfile

import pytest
import torch

from smdt_amd.models.hf import HFCausalLM, config_from_hf

transformers = pytest.importorskip("transformers")

CFGS = {
    "opt": dict(model_type="opt", hidden_size=64, num_hidden_layers=2, num_attention_heads=4, ffn_dim=128,
                vocab_size=100, max_position_embeddings=64, activation_function="relu", do_layer_norm_before=True,
                enable_bias=True, word_embed_proj_dim=64, pad_token_id=1, bos_token_id=2, eos_token_id=2),
    "llama": dict(model_type="llama", hidden_size=64, num_hidden_layers=2, num_attention_heads=4,
                  num_key_value_heads=2, intermediate_size=96, vocab_size=100, max_position_embeddings=64,
                  rms_norm_eps=1e-6, rope_theta=10000.0, hidden_act="silu", tie_word_embeddings=False,
                  bos_token_id=1, eos_token_id=2),
    "gpt2": dict(model_type="gpt2", n_embd=64, n_layer=2, n_head=4, vocab_size=100, n_positions=64,
                 activation_function="gelu_new", bos_token_id=0, eos_token_id=0),
}


@pytest.mark.parametrize("kind", sorted(CFGS))
def test_loss_and_logits_match_transformers(kind):
    torch.manual_seed(0)
    m = HFCausalLM(CFGS[kind], params_dtype=torch.float32).eval()
    ids = torch.randint(0, 100, (2, 16))
    labels = ids.clone()
    labels[:, :3] = -100  # prompt tokens masked like the SFT collator
    with tempfile.TemporaryDirectory() as d:
        m.save_pretrained(d)
        ref = transformers.AutoModelForCausalLM.from_pretrained(d, dtype=torch.float32,
                                                                attn_implementation="eager").eval()
        back = HFCausalLM.from_pretrained(d, params_dtype=torch.float32).eval()
    with torch.no_grad():
        r = ref(input_ids=ids, labels=labels)
        loss, _ = m(ids, labels=labels)
        loss2, _ = back(ids, labels=labels)
        _, logits = m(ids)
    torch.testing.assert_close(loss, r.loss, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(loss2, r.loss, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(logits, r.logits, rtol=1e-4, atol=1e-4)


def test_padded_vocab_excluded_from_loss():
    m = HFCausalLM(CFGS["opt"], params_dtype=torch.float32)
    assert m.cfg.padded_vocab_size == 128
    ids = torch.randint(0, 100, (1, 8))
    loss, _ = m(ids, labels=ids)
    loss.backward()
    g = m.model.embedding.weight.grad
    # padding rows get no gradient through the LM head (lookups never touch them either)
    assert g[100:].abs().max() == 0


def test_resize_token_embeddings_grows_padded_vocab():
    m = HFCausalLM(CFGS["llama"], params_dtype=torch.float32)
    m.resize_token_embeddings(130)
    assert m.vocab_size == 130 and m.cfg.padded_vocab_size == 256
    assert m.model.embedding.weight.shape[0] == 256 and m.model.output_weight.shape[0] == 256
    ids = torch.randint(0, 130, (1, 8))
    loss, _ = m(ids, labels=ids)
    assert torch.isfinite(loss)


def test_builtin_configs():
    from smdt_amd.models.hf import BUILTIN
    c = config_from_hf(BUILTIN["facebook/opt-125m"])
    assert (c.num_layers, c.hidden_size, c.activation, c.position_offset) == (12, 768, "relu", 2)
    c = config_from_hf(BUILTIN["llama-7b"])
    assert (c.num_layers, c.hidden_size, c.ffn_hidden_size, c.normalization) == (32, 4096, 11008, "RMSNorm")


def test_flash_dropout_mask_twin_properties():
    from smdt_amd.ops.functional import flash_dropout_keep_mask
    m1 = flash_dropout_keep_mask(2, 3, 128, 0.1, 42, 5)
    m2 = flash_dropout_keep_mask(2, 3, 128, 0.1, 42, 5)
    m3 = flash_dropout_keep_mask(2, 3, 128, 0.1, 42, 6)
    assert torch.equal(m1, m2) and not torch.equal(m1, m3)
    assert abs((1 - m1.float().mean().item()) - 0.1) < 0.01
    # heads and batches draw independent masks
    assert not torch.equal(m1[0, 0], m1[0, 1]) and not torch.equal(m1[0, 0], m1[1, 0])


@pytest.mark.gpu
def test_packed_rows_gather_kernel_matches_index_ops():
    """Padding-free micro-batches: attention's unpack ([T, 1, W] -> [L, b, W], zero pad rows) and
    pack ([L, b, C] -> [T, 1, C]) run as one row-gather kernel each way (gather_rows) — values and
    gradients equal torch's index_copy / index_select formulation."""
    import torch
    from smdt_amd.models import transformer as T
    torch.manual_seed(0)
    L, b = 37, 5
    lens = torch.tensor([37, 20, 5, 33, 1])
    pos = [s * b + bi for s in range(L) for bi in range(b) if s < lens[bi]]
    idx = torch.tensor(pos, dtype=torch.int64, device="cuda")
    W, C = 96, 64
    x = torch.randn(idx.numel(), 1, W, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    with T.packed_sequences(idx, b, L):
        u = T._unpack_rows(x)
        y = T._pack_rows(u[..., :C].contiguous() * 2)
    ref_u = x.new_zeros(L * b, W).index_copy(0, idx, x.detach().reshape(-1, W)).view(L, b, W)
    assert torch.equal(u.detach(), ref_u)
    torch.testing.assert_close(y.detach(), 2 * ref_u.reshape(-1, W)[idx][:, :C].unsqueeze(1))
    g = torch.randn_like(y)
    y.backward(g)
    gx = torch.zeros(idx.numel(), W, device="cuda", dtype=torch.bfloat16)
    gx[:, :C] = 2 * g.squeeze(1)
    torch.testing.assert_close(x.grad.squeeze(1), gx)


def test_length_groups_cost_gate():
    """The grouping is planned only when the attention work it saves pays for its extra launches:
    a LLaMA-7B-sized hidden groups an Alpaca-like window, an OPT-125m-sized one does not."""
    import torch
    from smdt_amd.models import transformer as T
    b, L = 32, 512
    g = torch.Generator().manual_seed(0)
    lens = torch.randint(40, 300, (b,), generator=g)
    lens[0] = 500
    mask = torch.arange(L).unsqueeze(0) < lens.unsqueeze(1)
    idx = torch.tensor(sorted(s * b + i for s in range(L) for i in range(b) if s < lens[i]), dtype=torch.int64)
    assert T.length_groups(mask, idx, "cpu", hidden=4096) is not None
    assert T.length_groups(mask, idx, "cpu", hidden=768) is None


def test_length_groups_plan_maps():
    """The length-grouped attention layout's host plan (models/transformer.length_groups): rows
    bucketed by their own length rounded up to 128, blocks [L_g, b_g] back to back; every real
    token sits at block offset + s * b_g + (its row's index in the block), the two maps invert
    each other, and a packed trailing pad token beyond its row's block maps to -1."""
    import torch
    from smdt_amd.models import transformer as T
    b, L = 5, 384
    lens = torch.tensor([300, 20, 130, 1, 128])
    mask = torch.arange(L).unsqueeze(0) < lens.unsqueeze(1)
    real = [s * b + i for s in range(L) for i in range(b) if s < lens[i]]
    extra = [200 * b + 1]                       # a pad position of row 1 (len 20, block 128)
    idx = torch.tensor(sorted(real + extra), dtype=torch.int64)
    g = T.length_groups(mask, idx, "cpu")
    assert [(Lg, bg) for _, Lg, bg in g["blocks"]] == [(128, 3), (256, 1), (384, 1)]
    assert g["rows"] == 128 * 3 + 256 + 384
    inv, pack = g["inv"], g["pack"]
    rows_of = {128: [1, 3, 4], 256: [2], 384: [0]}
    offs = {Lg: o for o, Lg, _ in g["blocks"]}
    for t, p in enumerate(idx.tolist()):
        s, i = p // b, p % b
        if s >= lens[i]:
            assert pack[t] == -1                 # the trailing pad beyond row 1's 128-block
            continue
        Lg = int(((int(lens[i]) + 127) // 128) * 128)
        j = rows_of[Lg].index(i)
        assert pack[t] == offs[Lg] + s * len(rows_of[Lg]) + j
        assert inv[pack[t]] == t
    assert int((inv >= 0).sum()) == len(real)


@pytest.mark.gpu
def test_length_grouped_attention_matches_padded_layout(monkeypatch):
    """Padding-free SFT micro-batch with attention in the length-grouped layout (blocks of rows
    of similar length, causal flash per block on views of one buffer) against the single padded
    [L, b] layout: the loss, every real token's loss and every parameter gradient agree (bf16,
    relative to each tensor's max), and the grouped path actually runs."""
    import torch
    from smdt_amd.models import transformer as T
    from smdt_amd.models.hf import HFCausalLM
    cfg = dict(model_type="llama", hidden_size=256, num_hidden_layers=2, num_attention_heads=4,
               num_key_value_heads=2, intermediate_size=512, vocab_size=120, max_position_embeddings=512,
               rms_norm_eps=1e-6, rope_theta=10000.0, tie_word_embeddings=False)
    torch.manual_seed(0)
    b, L = 6, 384
    lens = torch.tensor([300, 20, 130, 256, 5, 129])
    mask = (torch.arange(L).unsqueeze(0) < lens.unsqueeze(1)).long()
    ids = torch.randint(0, 120, (b, L))
    labels = torch.where(mask.bool(), ids, torch.full_like(ids, -100))
    calls = {"n": 0}
    orig = T.ParallelAttention._attend_groups

    def counted(self, *a):
        calls["n"] += 1
        return orig(self, *a)
    monkeypatch.setattr(T.ParallelAttention, "_attend_groups", counted)
    monkeypatch.setattr(T, "_GROUP_LAUNCH_S", 0.0)   # group even this small model (the cost gate)
    res = []
    for on in (True, False):
        monkeypatch.setattr(T, "_LENGTH_GROUPS", on)
        torch.manual_seed(1)
        m = HFCausalLM(cfg, params_dtype=torch.bfloat16, device="cuda")
        loss, tok = m(ids.cuda(), attention_mask=mask, labels=labels.cuda())
        loss.backward()
        res.append((loss.detach().float(), tok.detach().float(),
                    {n: p.grad.detach().float() for n, p in m.named_parameters() if p.grad is not None}))
    assert calls["n"] == 2                       # both layers, grouped run only
    (l1, t1, g1), (l0, t0, g0) = res
    assert abs(l1.item() - l0.item()) <= 1e-2 * abs(l0.item())
    real = mask.cuda().bool()
    assert (t1[real] - t0[real]).abs().max().item() <= 2e-2 * t0[real].abs().max().item()
    assert g1.keys() == g0.keys()
    for n in g0:
        assert (g1[n] - g0[n]).abs().max().item() <= 3e-2 * g0[n].abs().max().item() + 1e-6, n
