"""SFT path: Alpaca preprocessing, DeepSpeed-config resolution, ZeRO engine equivalence,
CPU-offload Adam, checkpoint/resume and zero_to_fp32 (reference
4_training_alpaca_deepspeed/train.py and configs/default_offload_opt_param.json)."""
import json
import os

import pytest
import torch

from smdt_amd.data import sft
from smdt_amd.train import hf_args
from smdt_amd.train.zero import resolve_ds_config

from _dist import run_workers  # noqa: E402
import dist_workers as W  # noqa: E402

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DS_CFG = os.path.join(REPO, "recipes", "4_training_alpaca_deepspeed", "configs", "default_offload_opt_param.json")
NB4 = ("--model_name_or_path facebook/opt-125m --data_path /opt/ml/input/data/training/alpaca_data.json "
       "--bf16 False --output_dir /opt/ml/model --num_train_epochs 1 --per_device_train_batch_size 4 "
       "--per_device_eval_batch_size 4 --gradient_accumulation_steps 8 --evaluation_strategy no "
       "--save_strategy steps --save_steps 2000 --save_total_limit 1 --learning_rate 2e-05 --weight_decay 0.0 "
       "--warmup_ratio 0.03 --deepspeed " + DS_CFG + " --tf32 False --cache_dir /opt/ml/input/data/cache_dir "
       "--report_to none").split()


def _parse(argv):
    p = hf_args.ArgumentParser((hf_args.ModelArguments, hf_args.DataArguments, hf_args.TrainingArguments))
    return p.parse_args_into_dataclasses(argv)


def test_nb4_cli_parses():
    m, d, t = _parse(NB4)
    assert m.model_name_or_path == "facebook/opt-125m"
    assert (t.per_device_train_batch_size, t.gradient_accumulation_steps, t.learning_rate) == (4, 8, 2e-5)
    assert t.bf16 is False and t.tf32 is False and t.save_total_limit == 1 and t.deepspeed == DS_CFG
    with pytest.raises(ValueError):
        _parse(NB4 + ["--no_such_flag", "1"])


def test_ds_auto_resolution_matches_hf_rules():
    _, _, t = _parse(NB4)
    raw = json.load(open(DS_CFG))
    cfg = resolve_ds_config(raw, t, hidden_size=768, world_size=16, num_training_steps=101)
    assert cfg["train_micro_batch_size_per_gpu"] == 4 and cfg["gradient_accumulation_steps"] == 8
    assert cfg["train_batch_size"] == 512                                   # NB4: 4 x 8 x 16
    assert cfg["gradient_clipping"] == 1.0
    assert cfg["optimizer"]["params"] == {"lr": 2e-5, "betas": [0.9, 0.999], "eps": 1e-8, "weight_decay": 0.0}
    sp = cfg["scheduler"]["params"]
    assert (sp["warmup_min_lr"], sp["warmup_max_lr"], sp["warmup_num_steps"], sp["total_num_steps"]) == \
        (0, 2e-5, 4, 101)                                                   # ceil(0.03 * 101) = 4
    z = cfg["zero_optimization"]
    assert z["reduce_bucket_size"] == 768 * 768
    assert z["stage3_prefetch_bucket_size"] == int(0.9 * 768 * 768)
    assert z["stage3_param_persistence_threshold"] == 7680                 # NB4:1629 threshold
    assert cfg["bf16"]["enabled"] is False


def test_ds_explicit_mismatch_raises():
    _, _, t = _parse(NB4)
    raw = json.load(open(DS_CFG))
    raw["train_micro_batch_size_per_gpu"] = 16
    with pytest.raises(ValueError, match="differ"):
        resolve_ds_config(raw, t, 768, 16, 101)


def test_preprocess_masks_prompt_and_collator_pads():
    tok = sft.load_tokenizer("facebook/opt-125m", model_max_length=64)
    assert len(tok) == 50265 and tok.pad_token_id == 1 and tok.eos_token == "</s>"
    data = [{"instruction": "Give three tips.", "input": "", "output": "Eat well. Sleep."},
            {"instruction": "Translate", "input": "hello world", "output": "hola mundo"}]
    src, tgt = sft.format_examples(data, tok.eos_token)
    assert src[0].endswith("### Response:") and "### Input:\nhello world" in src[1]
    d = sft.preprocess(src, tgt, tok)
    for ids, lab, s in zip(d["input_ids"], d["labels"], src):
        n_src = len(tok(s, return_tensors="pt").input_ids[0])
        assert (lab[:n_src] == sft.IGNORE_INDEX).all()
        assert torch.equal(lab[n_src:], ids[n_src:])
        assert ids[-1].item() == tok.eos_token_id
    col = sft.DataCollatorForSupervisedDataset(tok, pad_to_multiple_of=32)
    b = col([{"input_ids": i, "labels": l} for i, l in zip(d["input_ids"], d["labels"])])
    assert b["input_ids"].shape[1] % 32 == 0
    assert (b["labels"][b["input_ids"] == tok.pad_token_id] == -100).all()
    assert torch.equal(b["attention_mask"], b["input_ids"].ne(tok.pad_token_id))


def test_pad_to_multiple_does_not_change_loss():
    from smdt_amd.models.hf import HFCausalLM
    torch.manual_seed(0)
    m = HFCausalLM(W.SFT_LLAMA, params_dtype=torch.float32).eval()
    ids, lab = W.sft_batches(1, b=2, s=20)[0]
    with torch.no_grad():
        l1, _ = m(ids, labels=lab)
        ids2 = torch.cat([ids, torch.zeros(2, 12, dtype=torch.long)], 1)
        lab2 = torch.cat([lab, torch.full((2, 12), -100)], 1)
        l2, _ = m(ids2, labels=lab2)
    torch.testing.assert_close(l1, l2, rtol=1e-6, atol=1e-6)


def test_length_grouped_sampler_covers_dataset_once():
    lens = torch.randint(5, 300, (103,)).tolist()
    seen = []
    for r in range(2):
        s = sft.LengthGroupedSampler(lens, batch_size=4, rank=r, world=2, seed=1)
        seen += list(iter(s))
    assert sorted(set(seen)) == list(range(103))


def test_cpu_adam_matches_torch_adamw():
    from smdt_amd import _runtime
    torch.manual_seed(0)
    n = 100_003
    p = torch.randn(n)
    g = torch.randn(n)
    m = torch.zeros(n)
    v = torch.zeros(n)
    ref = p.clone().requires_grad_()
    opt = torch.optim.AdamW([ref], lr=1e-2, betas=(0.9, 0.95), eps=1e-8, weight_decay=0.1)
    out = torch.empty(n, dtype=torch.int16)
    for step in range(1, 4):
        ref.grad = g.clone() * 0.5
        opt.step()
        _runtime.cpu_adam(p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr(), out.data_ptr(), n, 1e-2, 0.9,
                          0.95, 1e-8, 0.1, step, True, 0.5, 4)
    torch.testing.assert_close(p, ref.detach(), rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(out.view(torch.bfloat16).float(), p.to(torch.bfloat16).float())


@pytest.mark.slow
@pytest.mark.parametrize("stage,ga,offload,offload_param", [
    (0, 1, False, False), (1, 1, False, False), (2, 1, False, False), (2, 2, False, False), (3, 1, False, False),
    (3, 2, False, False), (2, 1, True, False), (3, 1, True, True), (3, 1, False, True)])
def test_zero_world2_matches_world1(stage, ga, offload, offload_param):
    """Every ZeRO stage (2: partitioned gradients; 3: + partitioned parameters gathered per layer,
    optionally offloaded to pinned host memory, with CPU Adam) reproduces single-rank training."""
    # GA 2*ga on one rank, folded like two ranks (dist_workers._emulated_reference_steps)
    ref = run_workers(W.zero_sft_worker, 1, 0, 2 * ga, 3, False, False, False, False, 2, stage)[0]
    outs = run_workers(W.zero_sft_worker, 2, stage, ga, 3, offload, offload_param)   # GA ga on two ranks
    for r in range(2):
        for k, v in ref.items():
            _adam_close(outs[r][k], v, steps=3, what=(r, k))


@pytest.mark.parametrize("ga,tied", [(1, False), (2, False), (1, True), (2, True)])
def test_zero2_lazy_grad_buffers_match_world1(ga, tied, monkeypatch):
    """ZeRO-2 with dp 2 allocates each bucket's fp32 accumulation buffer uninitialised: the
    deferred wgrad launch stores the first gradient of a weight (no zero fill, no read), other
    writers zero their slice on first access, unwritten slices and alignment padding are zeroed
    before the reduce-scatter. Training equals single-rank training (CPU path of the queue). Tied:
    the word embedding's lookup gradient and the LM head's queued wgrad STORE share one slice —
    the lookup's write flushes the queue first."""
    monkeypatch.setenv("SMDT_TEST_CPU_DEFER", "1")
    if tied:
        monkeypatch.setenv("SMDT_TEST_TIED", "1")
    ref = run_workers(W.zero_sft_worker, 1, 0, 2 * ga, 3, False, False, False, False, 2, 2)[0]
    outs = run_workers(W.zero_sft_worker, 2, 2, ga, 3, False, False, True)
    for r in range(2):
        params, mem = outs[r]
        assert mem["wgrad_stats"]["stores"] > 0, mem["wgrad_stats"]    # the store path ran
        for k, v in ref.items():
            _adam_close(params[k], v, steps=3, what=(r, k))


@pytest.mark.slow
def test_zero2_world8_matches_world1():
    """ZeRO-2 over 8 gloo ranks (gradient shards of 1/8, one micro-batch each) == one rank
    accumulating the same 8 micro-batches."""
    ref = run_workers(W.zero_sft_worker, 1, 0, 8, 2, False, False, False, False, 8, 2)[0]
    outs = run_workers(W.zero_sft_worker, 8, 2, 1, 2, False, False, timeout=600)
    for r in range(8):
        for k, v in ref.items():
            _adam_close(outs[r][k], v, steps=2, what=(r, k))


def _adam_close(got, ref, steps, what, lr=1e-3):
    """Parameters after ``steps`` AdamW steps (eps 1e-8) agree elementwise at rtol 2e-4 / atol
    2e-5. The reference folds the micro-batch gradients in the sharded run's fixed order
    (dist_workers._emulated_reference_steps, DistributedDataParallel.deterministic_reduce), so the
    reduced gradients are equal; the gradient norm is accumulated in fp64 (optim/optimizer._sumsq)
    and does not depend on the shard split. What remains is the CPU-Adam / torch-Adam arithmetic
    of the offload configurations."""
    torch.testing.assert_close(got, ref, rtol=2e-4, atol=2e-5, msg=str(what))


@pytest.mark.parametrize("world", [2, 4])
def test_zero_stage3_memory_is_partitioned(world):
    """Per-rank persistent gradient and parameter storage ~ total / dp under ZeRO-3 (plus the small
    always-gathered buckets), and the model holds no full parameter between steps."""
    outs = run_workers(W.zero_sft_worker, world, 3, 1, 1, False, False, True)
    for _, mem in outs:
        total = mem["total"]
        assert mem["grad"] <= total / world * 1.05 + 4096, mem
        assert mem["param"]["shard"] <= total / world * 1.05 + 4096, mem
        assert mem["param"]["persistent"] < 0.05 * total, mem
        assert mem["param_numel_now"] <= mem["param"]["persistent"] + 4096, mem
        assert mem["wt_cache_left"] == 0, mem      # no dgrad W^T of a freed bucket survives


@pytest.mark.parametrize("world", [4])
def test_zero_init_partitioned_construction(world):
    """ZeRO-3 partitioned construction (parallel/zero_init.py, DeepSpeed zero.Init, VERDICT r2
    item 8): while the model is built a rank never holds more than its shards plus ONE full
    parameter, nothing full is resident afterwards, and training from it matches the resident
    build (and hence single-rank training) step for step."""
    ref = run_workers(W.zero_sft_worker, world, 3, 1, 2, False, False, True, False)
    outs = run_workers(W.zero_sft_worker, world, 3, 1, 2, False, False, True, True)
    for (params, mem), (rparams, rmem) in zip(outs, ref):
        ini = mem["init"]
        full_bytes = rmem["init"]["resident_bytes_after_build"]
        assert ini["params"] > 0 and ini["resident_bytes_after_build"] == 0, ini
        # peak = shards kept so far + the one parameter being cut (padding: < 1 element per rank/param)
        assert ini["peak_bytes"] <= full_bytes / world + ini["largest_param_bytes"] + 4 * ini["params"], ini
        assert ini["peak_bytes"] < 0.6 * full_bytes, (ini, full_bytes)
        assert mem["param"]["shard"] == rmem["param"]["shard"] and mem["grad"] == rmem["grad"]
        for k, v in rparams.items():
            torch.testing.assert_close(params[k], v, rtol=0, atol=0, msg=k)


def test_zero_init_stock_torch_modules():
    """nn.Linear / nn.LayerNorm / nn.Embedding and a module whose own constructor initialises its
    parameter, built under zero_init.Init at world 2, equal the resident build (the constructor
    finishes before the cut) and leave only shards behind."""
    for o in run_workers(W.zero_init_torch_modules_worker, 2):
        assert all(o["equal"].values()), o["equal"]
        assert o["params"] == 7 and o["resident"] == 0, o
        assert o["shard"] <= o["full"] / 2 + 4 * 7 and o["peak"] < o["full"], o


def test_zero_init_embedding_resize_stays_partitioned():
    for o in run_workers(W.zero_init_resize_worker, 2):
        assert o["part"] == [True, True] and o["same_objects"], o
        assert o["shape"] == [(256, 64), (256, 64)] and o["old_equal"] and o["new_rows"] == [7.0], o
        assert o["resident"] == 0, o


def _trainer_args(tmp_path, **over):
    argv = ["--output_dir", str(tmp_path / "out"), "--per_device_train_batch_size", "2",
            "--gradient_accumulation_steps", "2", "--learning_rate", "1e-3", "--logging_steps", "1",
            "--save_steps", "3", "--max_steps", "6", "--deepspeed", DS_CFG, "--pad_to_multiple_of", "8",
            "--warmup_steps", "2", "--seed", "5"]
    for k, v in over.items():
        argv += [f"--{k}", str(v)]
    return _parse(argv)[2]


def _tiny_trainer(tmp_path, args):
    from smdt_amd.models.hf import HFCausalLM
    from smdt_amd.parallel import state as ps
    from smdt_amd.train.sft_trainer import Trainer
    ps.destroy_model_parallel()
    torch.manual_seed(0)
    model = HFCausalLM(W.SFT_LLAMA, params_dtype=torch.float32)
    tok = sft.HashWordTokenizer(120, 48, pad_token="<pad>", special_ids={"<pad>": 0, "</s>": 1, "<s>": 2, "<unk>": 3})
    path = tmp_path / "alpaca.json"
    if not path.exists():
        sft.write_synthetic_alpaca(str(path), 40, seed=1)
    ds = sft.SupervisedDataset(str(path), tok)
    return Trainer(model=model, tokenizer=tok, args=args, train_dataset=ds,
                   data_collator=sft.DataCollatorForSupervisedDataset(tok, 8))


def test_trainer_checkpoint_resume_and_zero_to_fp32(tmp_path):
    from smdt_amd.train.zero import get_fp32_state_dict_from_zero_checkpoint
    t = _tiny_trainer(tmp_path, _trainer_args(tmp_path))
    met = t.train()
    with t.engine.gathered_params():            # ZeRO-3 (the reference config): params are partitioned
        full = {k: v.detach().clone() for k, v in t.model.named_parameters()}
    losses = [h["loss"] for h in t.state["log_history"] if "loss" in h]
    assert len(losses) == 6 and met["train_samples_per_second"] > 0
    ck = tmp_path / "out" / "checkpoint-6"
    assert (ck / "latest").read_text() == "global_step6"
    assert (ck / "global_step6" / "mp_rank_00_model_states.pt").exists()
    assert (tmp_path / "out" / "checkpoint-3").exists()
    sd = get_fp32_state_dict_from_zero_checkpoint(str(ck))
    for k, v in full.items():
        torch.testing.assert_close(sd["model." + k] if "model." + k in sd else sd[k], v)
    # resuming from the step-3 checkpoint reproduces the uninterrupted run
    t3 = _tiny_trainer(tmp_path, _trainer_args(tmp_path, output_dir=tmp_path / "out2",
                                               resume_from_checkpoint=tmp_path / "out" / "checkpoint-3"))
    t3.train()
    with t3.engine.gathered_params():
        got = {k: v.detach().clone() for k, v in t3.model.named_parameters()}
    for k, v in full.items():
        torch.testing.assert_close(got[k], v, rtol=1e-5, atol=1e-6)


def test_window_that_does_not_fit_runs_micro_batches(tmp_path, monkeypatch):
    """A fused accumulation window over the free-memory budget (Trainer._window_fits False) runs
    its micro-batches one by one: same losses and parameters as SMDT_SFT_FUSE_GA=0."""
    from smdt_amd.train.sft_trainer import Trainer
    runs = []
    for mode in ("off", "nofit"):
        if mode == "off":
            monkeypatch.setenv("SMDT_SFT_FUSE_GA", "0")
        else:
            monkeypatch.delenv("SMDT_SFT_FUSE_GA", raising=False)
            monkeypatch.setattr(Trainer, "_window_fits", lambda self, window: False)
        t = _tiny_trainer(tmp_path, _trainer_args(tmp_path, output_dir=tmp_path / mode, max_steps=3,
                                                  save_steps=0))
        t.train()
        with t.engine.gathered_params():
            runs.append(([h["loss"] for h in t.state["log_history"] if "loss" in h],
                         {k: v.detach().clone() for k, v in t.model.named_parameters()}))
    assert runs[0][0] == runs[1][0]
    for k, v in runs[0][1].items():
        torch.testing.assert_close(runs[1][1][k], v, rtol=0, atol=0)


def test_emulated_dp_rank_holds_one_shard(tmp_path, monkeypatch):
    """SMDT_EMULATE_DP=8: one process runs one ZeRO rank of an 8-GPU job (loopback DP group,
    comm/loopback.py): its gradient / optimizer storage is 1/8 of the model and the metrics name
    the emulation and the predicted job rate."""
    monkeypatch.setenv("SMDT_EMULATE_DP", "8")
    try:
        t = _tiny_trainer(tmp_path, _trainer_args(tmp_path, max_steps=2, save_steps=0,
                                                  deepspeed=os.path.join(REPO, "recipes", "4_training_alpaca_deepspeed", "configs", "zero2_bf16.json"),
                                                  bf16=False))
        met = t.train()
        ddp = t.engine.ddp
        total = sum(p.numel() for p in t.model.parameters())
        assert ddp.dp == 8 and ddp.grad_memory_numel() <= total / 8 * 1.05 + 4096
        assert met["emulated_dp_ranks"] == 8
        assert met["predicted_job_train_samples_per_second"] == pytest.approx(8 * met["train_samples_per_second"], rel=1e-3)
    finally:
        from smdt_amd.parallel import state as ps
        ps.destroy_model_parallel()


def test_save_total_limit_rotates(tmp_path):
    t = _tiny_trainer(tmp_path, _trainer_args(tmp_path, save_total_limit=1, save_steps=2))
    t.train()
    cks = sorted(p.name for p in (tmp_path / "out").iterdir() if p.name.startswith("checkpoint-"))
    assert cks == ["checkpoint-6"]


@pytest.mark.parametrize("mt", ["llama", "opt"])
def test_padding_free_microbatch_matches_padded(mt, monkeypatch):
    """A right-padded micro-batch run on its real tokens only (models/transformer.py
    packed_sequences: attention alone sees the padded layout) gives the padded run's loss,
    per-token losses and every gradient."""
    from smdt_amd.models.hf import HFCausalLM
    from smdt_amd.models import transformer as T
    if mt == "llama":
        cfg = W.SFT_LLAMA
    else:
        cfg = {"model_type": "opt", "hidden_size": 64, "num_hidden_layers": 2, "num_attention_heads": 4,
               "ffn_dim": 128, "max_position_embeddings": 128, "vocab_size": 120, "word_embed_proj_dim": 64,
               "do_layer_norm_before": True, "activation_function": "relu", "pad_token_id": 1, "enable_bias": True}
    torch.manual_seed(0)
    m = HFCausalLM(cfg, params_dtype=torch.float32).eval()
    b, L = 4, 64
    ids = torch.randint(3, 100, (b, L))
    am = torch.zeros(b, L, dtype=torch.bool)
    for i, n in enumerate([64, 40, 17, 9]):
        am[i, :n] = True
    ids[~am] = 0
    lab = ids.clone()
    lab[~am] = -100
    lab[:, :3] = -100
    monkeypatch.setenv("SMDT_SFT_UNPAD", "0")
    l0, t0 = m(ids, attention_mask=am, labels=lab)
    g0 = torch.autograd.grad(l0, list(m.parameters()))
    monkeypatch.setenv("SMDT_SFT_UNPAD", "1")
    calls = []
    orig = T._unpack_rows
    monkeypatch.setattr(T, "_unpack_rows", lambda x: calls.append(x.shape[0]) or orig(x))
    l1, t1 = m(ids, attention_mask=am, labels=lab)
    g1 = torch.autograd.grad(l1, list(m.parameters()))
    assert calls and calls[0] == 192                    # 130 real tokens rounded up to 64 with pads
    torch.testing.assert_close(l1, l0, rtol=1e-6, atol=1e-6)
    keep = torch.zeros_like(am)
    keep[:, :-1] = lab[:, 1:] != -100
    torch.testing.assert_close(t1[keep], t0[keep], rtol=1e-5, atol=1e-6)
    for a, c in zip(g0, g1):
        torch.testing.assert_close(c, a, rtol=1e-4, atol=1e-6)


def test_fused_accumulation_window_matches_micro_batches():
    """SFT trainer's fused GA window (train/sft_trainer._fuse_window + HFCausalLM row_groups +
    ZeroEngine.backward(window=True)): one batch carrying GA right-padded micro-batches of
    different lengths gives the same losses and parameters as GA accumulated micro-batches."""
    import dist_workers as W
    from smdt_amd.models.hf import HFCausalLM
    from smdt_amd.parallel import state as ps
    from smdt_amd.train.sft_trainer import _fuse_window
    from smdt_amd.train.zero import ZeroEngine
    ga, steps = 4, 2
    g = torch.Generator().manual_seed(5)
    micro = []
    for i in range(ga * steps):
        L = 10 + 2 * (i % 3)
        ids = torch.randint(1, 120, (2, L), generator=g)
        mask = torch.ones(2, L, dtype=torch.bool)
        mask[1, L - 3:] = False                      # right padding in the second row
        lab = ids.clone()
        lab[:, :3] = -100
        lab[~mask] = -100
        micro.append(dict(input_ids=ids, labels=lab, attention_mask=mask))
    cfg = {"optimizer": {"type": "AdamW", "params": {"lr": 1e-3, "weight_decay": 0.0}},
           "gradient_accumulation_steps": ga, "gradient_clipping": 1.0, "zero_optimization": {"stage": 2}}
    runs = []
    for fused in (False, True):
        ps.destroy_model_parallel()
        torch.manual_seed(0)
        m = HFCausalLM(W.SFT_LLAMA, params_dtype=torch.float32)
        eng = ZeroEngine(m, cfg, log=lambda *_: None)
        losses = []
        for s in range(steps):
            win = micro[s * ga:(s + 1) * ga]
            if fused:
                b, groups = _fuse_window(win)
                loss, _ = m(b["input_ids"], attention_mask=b["attention_mask"], labels=b["labels"], row_groups=groups)
                eng.backward(loss, window=True)
                losses.append(float(loss.detach()))
                assert eng.step() is not None
            else:
                tot = 0.0
                for b in win:
                    loss, _ = m(b["input_ids"], attention_mask=b["attention_mask"], labels=b["labels"])
                    eng.backward(loss)
                    tot += float(loss.detach()) / ga
                    gn = eng.step()
                losses.append(tot)
                assert gn is not None
        runs.append((losses, {n: p.detach().clone() for n, p in m.named_parameters()}))
    (l0, p0), (l1, p1) = runs
    assert abs(l0[0] - l1[0]) < 1e-5 and abs(l0[1] - l1[1]) < 1e-4, (l0, l1)
    for n in p0:
        torch.testing.assert_close(p1[n], p0[n], atol=1e-5, rtol=1e-4, msg=n)


@pytest.mark.parametrize("cfg", ["zero2_bf16.json", "default_offload_opt_param.json"])
def test_fused_window_decision_agreed_across_ranks(tmp_path, cfg):
    """Only rank 1 finds its fused accumulation window too large: both ranks must run the window
    micro-batch by micro-batch (ZeRO-2 reduce-scatters per micro-batch, ZeRO-3 gathers per
    forward, so a split decision hangs or mis-reduces). Result equals SMDT_SFT_FUSE_GA=0."""
    ds = os.path.join(REPO, "recipes", "4_training_alpaca_deepspeed", "configs", cfg)
    split = run_workers(W.sft_window_agreement_worker, 2, str(tmp_path), ds, 1, True, timeout=400)
    off = run_workers(W.sft_window_agreement_worker, 2, str(tmp_path), ds, -1, False, timeout=400)
    assert not any("fused accumulation window:" in m for _, logs in split for m in logs)
    assert any("would not fit" in m for m in split[0][1])          # rank 0 fits alone, yet agrees
    # Both ranks hold the same gathered result; it equals the unfused run up to fp32 summation
    # order: ZeRO-2's per-micro-batch reduce-scatters overlap the backward, and under a loaded
    # parallel test run their landing order moved gradient ulps (Adam turns a near-zero gradient's
    # ulp flip into an lr-sized step, so a few elements differ by up to 2 x lr after 2 steps).
    for k, v in off[0][0].items():
        torch.testing.assert_close(split[1][0][k], split[0][0][k], rtol=0, atol=0)
        d = (split[0][0][k].float() - v.float()).abs()
        assert d.max() <= 2.5e-3 and (d <= 1e-6).float().mean() >= 0.9, (k, d.max().item())


def test_zero_init_contexts_nest_and_restore_init_subclass():
    """Nested Init contexts: the inner exit must not drop the outer hook, the outer
    exit must not raise, and an __init_subclass__ another library put on nn.Module survives."""
    from torch import nn
    from smdt_amd.parallel import zero_init as zi
    seen = []

    def lib_hook(cls, **kw):
        seen.append(cls.__name__)
    nn.Module.__init_subclass__ = classmethod(lib_hook)
    try:
        with zi.Init(enabled=True):
            with zi.Init(enabled=True):
                class A(nn.Module):
                    pass
            class B(nn.Module):          # outer context still hooks new classes
                pass
        class C(nn.Module):
            pass
        assert seen == ["A", "B", "C"]
        assert nn.Module.__dict__["__init_subclass__"].__func__ is lib_hook
    finally:
        del nn.Module.__init_subclass__
    assert "__init_subclass__" not in nn.Module.__dict__
