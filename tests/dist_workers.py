"""Worker bodies for the multi-process (gloo, CPU) tests. Importable by spawned children."""
import os
import time
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

TINY = dict(num_layers=2, hidden_size=64, num_attention_heads=4, max_position_embeddings=32,
            padded_vocab_size=128, hidden_dropout=0.0, attention_dropout=0.0, params_dtype=torch.float32,
            use_flash_attn=True, seed=7)


def _batch(seed=0, b=4, s=32, v=128):
    g = torch.Generator().manual_seed(seed)
    toks = torch.randint(0, v, (b, s + 1), generator=g)
    return toks[:, :-1].contiguous(), toks[:, 1:].contiguous()


def gpt_reference(steps=1, sp=False, cfg_over=None):
    """Single-process TP=1 run: per-token loss + named full gradients."""
    from smdt_amd.models.gpt import GPTModel
    from smdt_amd.models.transformer import TransformerConfig
    from smdt_amd.parallel import state as ps
    ps.destroy_model_parallel()
    cfg = TransformerConfig(**{**TINY, **(cfg_over or {})})
    m = GPTModel(cfg)
    tokens, labels = _batch()
    loss = m(tokens, None, None, labels=labels)
    loss.mean().backward()
    grads = {n: p.grad.detach().clone() for n, p in m.named_parameters() if p.grad is not None}
    return loss.detach(), grads


class _Done:
    def wait(self):
        return True


class _GlooPieceEngine:
    """CPU stand-in of the xGMI engine's piece API (comm/xgmi.XgmiAllReduce.all_gather_pieces_async
    / reduce_scatter_piece_async) over a Gloo group, synchronous: lets the Gloo equivalence tests
    run ``TpDirect``'s row-piece logic and every ring caller's row-range / write-into-``out``
    callbacks. Reductions sum in rank order, as the engine does."""

    def __init__(self, group):
        import torch.distributed as dist
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.active = True
        self.use = {"all_gather": True, "reduce_scatter": True}

    def all_gather_pieces_async(self, flat, stride, ranges):
        import torch.distributed as dist
        hs = []
        for lo, hi in ranges:
            mine = flat[self.rank * stride + lo:self.rank * stride + hi].clone()
            parts = [torch.empty_like(mine) for _ in range(self.world)]
            dist.all_gather(parts, mine, group=self.group)
            for r in range(self.world):
                flat[r * stride + lo:r * stride + hi].copy_(parts[r])
            hs.append(_Done())
        return hs

    def reduce_scatter_piece_async(self, out, inp, lo, hi, stride):
        import torch.distributed as dist
        mine = torch.cat([inp[d * stride + lo:d * stride + hi] for d in range(self.world)])
        parts = [torch.empty_like(mine) for _ in range(self.world)]
        dist.all_gather(parts, mine, group=self.group)
        n = hi - lo
        acc = parts[0][self.rank * n:(self.rank + 1) * n].clone()
        for r in range(1, self.world):
            acc += parts[r][self.rank * n:(self.rank + 1) * n]
        out[lo:hi].copy_(acc)
        return _Done()


def _cpu_tp_direct(group, pieces):
    """A ``TpDirect`` over ``_GlooPieceEngine`` that accepts CPU tensors."""
    from smdt_amd.comm import tp_direct

    class _CpuTpDirect(tp_direct.TpDirect):
        def fits(self, t):
            return self.active and t.numel() > 0 and (t.numel() * t.element_size()) % 16 == 0

    tp_direct.PIECES = pieces
    return _CpuTpDirect(_GlooPieceEngine(group), group)


def gpt_tp_worker(rank, world, tp, pp, sp, cfg_over=None, p2p=None, direct_pieces=0, subbatch=0, ring_pieces=1):
    """``direct_pieces`` > 0: the TP exchanges run through ``TpDirect`` in that many row pieces
    (over the CPU stand-in engine) instead of the ring. ``subbatch`` = 2: the layer stack runs the
    two batch halves interleaved phase by phase (SMDT_SP_SUBBATCH)."""
    import torch.distributed as dist
    from smdt_amd.comm import init_distributed
    from smdt_amd.models.gpt import GPTModel, allreduce_word_embedding_grads
    from smdt_amd.models.transformer import TransformerConfig
    from smdt_amd.parallel import state as ps
    from smdt_amd.train.schedules import get_forward_backward_func
    init_distributed("gloo")
    st = ps.initialize_model_parallel(tp, pp)
    if ring_pieces > 1:
        from smdt_amd.parallel import tensor_parallel as _TPr
        _TPr._RING_PIECES = ring_pieces
    if subbatch:
        import smdt_amd.models.transformer as T
        T._SUBBATCH = subbatch
    if direct_pieces:
        st.tp_direct = _cpu_tp_direct(st.tp_group, direct_pieces)
    from smdt_amd.train import schedules
    schedules.configure_p2p(**(p2p or {}))
    cfg = TransformerConfig(**{**TINY, **(cfg_over or {}), "sequence_parallel": sp})
    m = GPTModel(cfg, pre_process=st.is_first_stage(), post_process=st.is_last_stage())
    tokens, labels = _batch()
    if pp == 1:
        loss = m(tokens, None, None, labels=labels)
        loss.mean().backward()
        out_loss = loss.detach()
    else:
        it = iter([(tokens, labels)] * 4)
        mb = 2
        toks_mb = tokens.chunk(2)
        labs_mb = labels.chunk(2)
        data = iter(list(zip(toks_mb, labs_mb)))

        def fstep(di, model):
            t, l = next(di)
            o = model(t, None, None, labels=l)

            def lf(x):
                return x.mean(), {"loss": x.detach()}
            return o, lf
        fb = get_forward_backward_func()
        seq = 32 // tp if sp else 32
        res = fb(fstep, data, m, 2, tensor_shape=(seq, mb, 64), dtype=torch.float32)
        allreduce_word_embedding_grads(m)
        out_loss = torch.cat([r["loss"] for r in res]) if res else None
    grads = {n: p.grad.detach().clone() for n, p in m.named_parameters() if p.grad is not None}
    # sequence-parallel replicated params: sum partial grads over TP (what the DDP wrapper does)
    if sp and tp > 1:
        for n, p in m.named_parameters():
            if getattr(p, "sequence_parallel", False) and n in grads:
                dist.all_reduce(grads[n], group=st.tp_group)
    meta = {"tp_rank": st.tp_rank, "pp_rank": st.pp_rank, "first": st.first_layer if hasattr(st, "first_layer") else None,
            "layer_offset": m.first_layer,
            "direct_calls": st.tp_direct.calls if direct_pieces else 0,
            "direct_pieces": st.tp_direct.pieces_issued if direct_pieces else 0}
    from smdt_amd.parallel import tensor_parallel as TPm
    meta["split"] = dict(TPm.SPLIT_STATS)
    dist.destroy_process_group()
    return out_loss, grads, meta


def ddp_worker(rank, world, zero, steps=3, overlap_pg=False, defer=False):
    """DDP (+ZeRO) on a tiny GPT: returns final params after `steps` optimizer steps on a
    per-rank shard of a fixed global batch (so the result must equal single-process training on
    the whole batch). ``defer``: weight gradients go through the deferred grouped-wgrad queue
    (CPU fallback), flushed every couple of GEMMs so buckets become ready mid-backward."""
    import torch.distributed as dist
    from smdt_amd.comm import init_distributed
    from smdt_amd.models.gpt import GPTModel
    from smdt_amd.models.transformer import TransformerConfig
    from smdt_amd.optim.optimizer import MixedPrecisionAdam
    from smdt_amd.parallel import state as ps
    from smdt_amd.parallel.distributed import DistributedDataParallel
    init_distributed("gloo")
    ps.initialize_model_parallel(1, 1)
    if defer:
        from smdt_amd.parallel import tensor_parallel as tp
        tp.DEFERRED_WGRAD.allow_cpu = True
        tp.DEFERRED_WGRAD.flush_tiles = 2
    cfg = TransformerConfig(**TINY)
    m = GPTModel(cfg)
    ddp = DistributedDataParallel(m, bucket_size=20000, use_distributed_optimizer=zero,
                                  overlap_param_gather=overlap_pg)
    opt = MixedPrecisionAdam(ddp, lr=1e-2, weight_decay=0.1, clip_grad=1.0, eps=1e-8)
    tokens, labels = _batch(b=4)
    shard = slice(rank * (4 // world), (rank + 1) * (4 // world))
    first_grads = None
    for _ in range(steps):
        ddp.zero_grad_buffer()
        loss = ddp(tokens[shard], None, None, labels=labels[shard]).mean()
        loss.backward()
        ddp.finish_grad_sync()
        if first_grads is None:
            if zero:  # only this rank's shard of each bucket is reduced: gather for comparison
                full = ddp.grad_data.clone()
                for b in ddp.buckets:
                    s, e = ddp.shard_range(b)
                    dist.all_gather_into_tensor(full[b.start:b.end], ddp.grad_data[s:e].clone())
            else:
                full = ddp.grad_data.clone()
            first_grads = {n: full[ddp.param_index[id(p)][0]:ddp.param_index[id(p)][0] + p.numel()].view_as(p).clone()
                           for n, p in m.named_parameters()}
        opt.step()
    ddp.wait_param_gather()
    out = {n: p.detach().clone() for n, p in m.named_parameters()}
    dist.destroy_process_group()
    return out, first_grads


def single_train(steps=3, split=2):
    """Single-process reference for ``ddp_worker``: the global batch of 4 sequences as ``split``
    (the DP world size) micro-batches whose gradients land in separate buffers and are then
    combined in rank order and divided by ``split`` — the association the reduced run uses
    ((g_0 + g_1) / 2 over two ranks, exact up to that fixed order), so the reduced gradients are
    bit-identical and Adam runs at its real eps 1e-8 (a near-zero gradient summed in another
    order would flip its step-1 update sign, an lr-sized parameter difference)."""
    from smdt_amd.models.gpt import GPTModel
    from smdt_amd.models.transformer import TransformerConfig
    from smdt_amd.optim.optimizer import MixedPrecisionAdam
    from smdt_amd.parallel import state as ps
    from smdt_amd.parallel.distributed import DistributedDataParallel
    ps.destroy_model_parallel()
    cfg = TransformerConfig(**TINY)
    m = GPTModel(cfg)
    ddp = DistributedDataParallel(m, bucket_size=20000)
    opt = MixedPrecisionAdam(ddp, lr=1e-2, weight_decay=0.1, clip_grad=1.0, eps=1e-8)
    tokens, labels = _batch(b=4)
    first_grads = None
    per = 4 // split
    for _ in range(steps):
        parts = []
        for k in range(split):
            ddp.zero_grad_buffer()
            sl = slice(k * per, (k + 1) * per)
            loss = ddp(tokens[sl], None, None, labels=labels[sl]).mean()
            loss.backward()
            ddp.finish_grad_sync()
            parts.append(ddp.grad_data.clone())
        tot = parts[0]
        for p_ in parts[1:]:
            tot = tot + p_
        ddp.grad_data.copy_(tot * (1.0 / split))
        if first_grads is None:
            first_grads = {n: p.main_grad.detach().clone() for n, p in m.named_parameters()}
        opt.step()
    return {n: p.detach().clone() for n, p in m.named_parameters()}, first_grads


def mnist_ddp_worker(rank, world, data_dir, model_dir):
    os.environ["SM_MODEL_DIR"] = model_dir
    os.environ["SM_CHANNEL_TRAINING"] = data_dir
    sys.path.insert(0, os.path.join(ROOT, "recipes", "1_training_mnist_ddp"))
    import pytorch_mnist_ddp
    acc = pytorch_mnist_ddp.main(["--epochs", "1", "--backend", "gloo", "--log-interval", "20", "--save-model"])
    return acc


# ---------------------------------------------------------------------------------- SFT / ZeRO
SFT_LLAMA = dict(model_type="llama", hidden_size=64, num_hidden_layers=2, num_attention_heads=4,
                 num_key_value_heads=2, intermediate_size=96, vocab_size=120, max_position_embeddings=64,
                 rms_norm_eps=1e-6, rope_theta=10000.0, tie_word_embeddings=False)


def sft_batches(n=8, b=2, s=16, v=120, seed=3):
    g = torch.Generator().manual_seed(seed)
    out = []
    for _ in range(n):
        ids = torch.randint(0, v, (b, s), generator=g)
        lab = ids.clone()
        lab[:, :4] = -100
        out.append((ids, lab))
    return out


def zero_sft_worker(rank, world, stage, ga, steps, offload=False, offload_param=False, with_mem=False,
                    zero_init=False, emulate=0, emulate_stage=0):
    """Data-parallel SFT steps with the ZeroEngine; global batch = world * 2 * ga rows of
    ``sft_batches``. Returns full params after ``steps`` optimizer steps. ``zero_init``: build the
    model under parallel/zero_init.Init (stage 3).

    Multi-rank runs use the fixed-order combine (DistributedDataParallel ``deterministic_reduce``:
    rank-order sum, then / dp). ``emulate`` = W (world 1, ``ga`` = W x the emulated per-rank GA):
    the single-process reference reproduces that association exactly — each emulated rank's
    micro-batch gradients land in their own buffer and are folded in rank order, per
    accumulation window for gradient stages <= 1 (``emulate_stage``; each rank sums its window
    locally, then one reduction) or per micro-batch for stages >= 2 (reduced every micro-batch,
    accumulated into the shard) — so the runs agree bit for bit and Adam runs at its real eps."""
    from smdt_amd.comm import init_distributed
    from smdt_amd.models.hf import HFCausalLM
    from smdt_amd.parallel import state as ps
    from smdt_amd.parallel import zero_init as zi
    from smdt_amd.train.zero import ZeroEngine
    ps.destroy_model_parallel()
    init_distributed("gloo")
    ps.initialize_model_parallel(1, 1)
    from smdt_amd.parallel import tensor_parallel as _tpq
    if os.environ.get("SMDT_TEST_CPU_DEFER") == "1":
        # the weight gradients go through the deferred grouped-wgrad queue (CPU fallback): with
        # ZeRO-2's lazily zeroed staging buffers the first gradient of a weight is STORED
        _tpq.DEFERRED_WGRAD.allow_cpu = True
    torch.manual_seed(0)
    cfg_hf = SFT_LLAMA
    if os.environ.get("SMDT_TEST_TIED") == "1":     # tied LM head / word embedding (OPT, GPT-2 style)
        cfg_hf = dict(SFT_LLAMA, tie_word_embeddings=True)
    with zi.Init(enabled=zero_init) as ctx:
        m = HFCausalLM(cfg_hf, params_dtype=torch.float32)
    init_stats = {"peak_bytes": ctx.peak_bytes, "shard_bytes": ctx.shard_bytes, "params": ctx.params,
                  "largest_param_bytes": ctx.largest_param_bytes,
                  "resident_bytes_after_build": sum(p.numel() * p.element_size() for p in m.parameters())}
    if world > 1:
        os.environ["SMDT_DETERMINISTIC_REDUCE"] = "1"
    cfg = {"optimizer": {"type": "AdamW", "params": {"lr": 1e-3, "betas": [0.9, 0.99], "eps": 1e-8,
                                                     "weight_decay": 0.1}},
           "gradient_accumulation_steps": ga, "gradient_clipping": 1.0,
           "zero_optimization": {"stage": stage, **({"offload_optimizer": {"device": "cpu"}} if offload else {}),
                                 **({"offload_param": {"device": "cpu"}} if offload_param else {}),
                                 "stage3_param_persistence_threshold": 200, "stage3_prefetch_bucket_size": 4000}}
    eng = ZeroEngine(m, cfg, log=lambda *_: None)
    data = sft_batches(n=steps * ga * world + 8)
    if emulate > 1:
        _emulated_reference_steps(eng, m, data, emulate, ga // emulate, steps, emulate_stage)
    k = 0
    for _ in range(steps if emulate <= 1 else 0):
        for _ in range(ga):
            # each optimizer step consumes world*ga micro-batches in order; rank r takes every world-th
            ids = torch.cat([data[k + j * world + rank][0] for j in range(1)])
            lab = torch.cat([data[k + j * world + rank][1] for j in range(1)])
            k += world
            if stage == 3 and with_mem and k == steps * ga * world:     # before the last micro-batch
                # stand-in dgrad W^T entries (the cache only fills on GPU): a bucket freed by
                # the partitioner must drop its parameters' entries
                from smdt_amd.parallel import tensor_parallel as _tpm
                for p in m.parameters():
                    _tpm._WT_CACHE[id(p)] = (None, torch.empty(1))
            loss, _ = m(ids, labels=lab)
            eng.backward(loss * world / world)
            eng.step()
    eng.wait_for_params()
    wt_left = None
    if stage == 3 and with_mem:
        from smdt_amd.parallel import tensor_parallel as _tpm
        part = eng.partitioner
        wt_left = sum(1 for b in eng.ddp.buckets if not part.persistent[b.index]
                      for p in b.params if id(p) in _tpm._WT_CACHE)
        _tpm.params_changed()
    total = sum(eng.ddp.shapes[id(p)][0].numel() if hasattr(eng.ddp.shapes[id(p)][0], "numel")
                else int(torch.tensor(eng.ddp.shapes[id(p)][0]).prod()) for p in eng.ddp.params)
    mem = {"total": total, "grad": eng.ddp.grad_memory_numel(),
           "param": (eng.partitioner.param_memory_numel() if eng.partitioner is not None else None),
           "param_numel_now": sum(p.numel() for p in m.parameters()), "init": init_stats,
           "wt_cache_left": wt_left, "wgrad_stats": dict(_tpq.DEFERRED_WGRAD.stats)}
    with eng.gathered_params():
        out = {n: p.detach().clone() for n, p in m.named_parameters()}
    return (out, mem) if with_mem else out


def _emulated_reference_steps(eng, m, data, W, ga_r, steps, stage):
    """zero_sft_worker's ``emulate`` path: one process, W emulated ranks of ``ga_r`` micro-batches
    each per optimizer step (micro-batch j of rank r = data[base + j W + r], as in the W-rank run),
    gradients combined in the fixed order DistributedDataParallel.deterministic_reduce uses. The
    engine's GA is W ga_r, so each micro-batch loss carries 1 / (W ga_r) — the W-rank run's
    1 / ga_r and its / W after the rank-order sum, equal up to exact powers of two."""
    ddp = eng.ddp
    eng._hold_wgrad = lambda: False          # every micro-batch's gradient must land in the buffer

    def grad_of(idx):
        ddp.zero_grad_buffer()
        loss, _ = m(data[idx][0], labels=data[idx][1])
        eng.backward(loss)
        return ddp.grad_data.clone()

    base = 0
    for _ in range(steps):
        order = [(j, r) for r in range(W) for j in range(ga_r)] if stage <= 1 else \
            [(j, r) for j in range(ga_r) for r in range(W)]
        grads = {}
        for n_done, (j, r) in enumerate(order):
            grads[(j, r)] = grad_of(base + j * W + r)
            if n_done < len(order) - 1:
                eng.step()                    # not a boundary: counts the micro-batch
        if stage <= 1:                        # each rank sums its window, then the rank fold
            per_rank = []
            for r in range(W):
                acc = grads[(0, r)]
                for j in range(1, ga_r):
                    acc = acc + grads[(j, r)]
                per_rank.append(acc)
            tot = per_rank[0]
            for r in range(1, W):
                tot = tot + per_rank[r]
        else:                                 # reduced per micro-batch, accumulated into the shard
            tot = None
            for j in range(ga_r):
                f = grads[(j, 0)]
                for r in range(1, W):
                    f = f + grads[(j, r)]
                tot = f if tot is None else tot + f
        ddp.grad_data.copy_(tot)
        eng.step()                            # the boundary: optimizer step on the folded gradient
        base += W * ga_r


def zero_init_torch_modules_worker(rank, world):
    """Stock torch modules (their own reset_parameters() runs in the constructor) built under
    parallel/zero_init.Init over ``world`` gloo ranks: the gathered values equal a resident build
    from the same seed, and nothing full stays resident (Init used to cut a parameter at
    registration, before nn.Linear's init ran)."""
    import torch.nn as nn
    from smdt_amd.comm import init_distributed
    from smdt_amd.parallel import zero_init as zi
    init_distributed("gloo")

    class Block(nn.Module):
        def __init__(self):
            super().__init__()
            self.fc = nn.Linear(16, 12)
            self.norm = nn.LayerNorm(12)
            self.scale = nn.Parameter(torch.empty(12))
            nn.init.uniform_(self.scale, 0.5, 1.5)     # the owner's init code writes the full tensor

    def build():
        torch.manual_seed(3)
        return nn.ModuleList([nn.Embedding(10, 16), Block(), nn.Linear(12, 7, bias=False)])
    ref = build()
    with zi.Init() as ctx:
        got = build()
    out = {"params": ctx.params, "resident": sum(p.numel() for p in got.parameters()),
           "peak": ctx.peak_bytes, "shard": ctx.shard_bytes,
           "full": sum(p.numel() * p.element_size() for p in ref.parameters()), "equal": {}}
    for (n, p), (_, q) in zip(ref.named_parameters(), got.named_parameters()):
        out["equal"][n] = bool(torch.equal(zi.gather_full(q).view(p.shape), p.detach()))
    return out


def zero_init_resize_worker(rank, world):
    """The Alpaca recipe's embedding resize on a model built under zero_init.Init (inside
    ``gathered``): afterwards the GROWN embedding and LM head are partitioned, with the
    old rows kept and the new ones set by the block."""
    from smdt_amd.comm import init_distributed
    from smdt_amd.models.hf import HFCausalLM
    from smdt_amd.parallel import state as ps
    from smdt_amd.parallel import zero_init as zi
    ps.destroy_model_parallel()
    init_distributed("gloo")
    ps.initialize_model_parallel(1, 1)
    torch.manual_seed(0)
    ref = HFCausalLM(SFT_LLAMA, params_dtype=torch.float32)
    torch.manual_seed(0)
    with zi.Init():
        m = HFCausalLM(SFT_LLAMA, params_dtype=torch.float32)
    emb, head = m.model.embedding.weight, m.model.output_weight
    old_rows = 120                        # (rows 120.. are padding, overwritten below)
    with zi.gathered([emb, head]):
        m.resize_token_embeddings(130)
        emb.data[120:130] = 7.0
    return {"part": [zi.is_partitioned(emb), zi.is_partitioned(head)],
            "shape": [zi.logical_shape(emb), zi.logical_shape(head)],
            "same_objects": emb is m.model.embedding.weight and head is m.model.output_weight,
            "old_equal": bool(torch.equal(zi.gather_full(emb).view(-1, 64)[:old_rows], ref.model.embedding.weight.detach()[:old_rows])),
            "new_rows": zi.gather_full(emb).view(-1, 64)[120:130].unique().tolist(),
            "resident": sum(p.numel() for p in m.parameters())}


def gpt_vpp_worker(rank, world, nmb, p2p=None):
    """Interleaved pipeline (pp=2, vpp=2 chunks of 1 layer each, 4 layers): returns the last
    stage's per-token losses and every local gradient keyed by its single-model name."""
    import torch.distributed as dist
    import torch.nn as nn
    from smdt_amd.comm import init_distributed
    from smdt_amd.models.gpt import GPTModel, allreduce_word_embedding_grads
    from smdt_amd.models.transformer import TransformerConfig
    from smdt_amd.parallel import state as ps
    from smdt_amd.train.schedules import get_forward_backward_func
    init_distributed("gloo")
    st = ps.initialize_model_parallel(1, 2, 2)
    from smdt_amd.train import schedules
    schedules.configure_p2p(**(p2p or {}))
    cfg = TransformerConfig(**{**TINY, "num_layers": 4})
    chunks = []
    for c in range(2):
        st.virtual_pp_rank = c
        chunks.append(GPTModel(cfg, pre_process=st.is_first_stage(), post_process=st.is_last_stage()))
    st.virtual_pp_rank = 0
    model = nn.ModuleList(chunks)
    tokens, labels = _batch()
    data = iter(list(zip(tokens.chunk(nmb), labels.chunk(nmb))))

    def fstep(di, m):
        t, l = next(di)
        o = m(t, None, None, labels=l)
        return o, (lambda x: (x.mean(), {"loss": x.detach()}))

    fb = get_forward_backward_func()
    res = fb(fstep, data, model, nmb, tensor_shape=(32, 4 // nmb, 64), dtype=torch.float32)
    allreduce_word_embedding_grads(model)
    grads = {}
    for m in chunks:
        for n, p in m.named_parameters():
            if p.grad is None:
                continue
            name = n
            if n.startswith("decoder.layers."):
                parts = n.split(".")
                parts[2] = str(int(parts[2]) + m.first_layer)
                name = ".".join(parts)
            if n == "output_weight":
                name = "embedding.weight"
            grads[name] = p.grad.detach().clone()
    loss = torch.cat([r["loss"] for r in res]) if res else None
    dist.destroy_process_group()
    return loss, grads


def xgmi_ipc_worker(rank, world, port, outdir):
    """One rank of the cross-PROCESS test: real HIP-IPC handle exchange and peer mappings, all
    ranks on cuda:0 (a gloo group carries the handles; the all-reduce itself is the kernel)."""
    import os
    import pickle
    import traceback

    import torch
    from smdt_amd.comm import xgmi

    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "RANK": str(rank),
                       "WORLD_SIZE": str(world)})
    res = {"ok": [], "err": None, "error_word": None}
    try:
        import torch.distributed as dist
        dist.init_process_group("gloo", rank=rank, world_size=world)
        torch.cuda.set_device(0)
        eng = xgmi.XgmiAllReduce(None, region_bytes=16 << 20, blocks=32, validate=False)
        # one-shot (<= 4 MiB at world 2) and two-shot sizes in both dtypes
        for n, dtype in ((4096, torch.float32), (1 << 21, torch.float32), (3 << 20, torch.bfloat16),
                         (8192, torch.bfloat16)):
            for rep in range(3):
                base = torch.arange(n, device="cuda", dtype=torch.float32) % 97 + rep
                x = (base + 1000.0 * rank).to(dtype)
                ref = (base + 0.0).to(dtype).float()
                for r in range(1, world):
                    ref = ref + (base + 1000.0 * r).to(dtype).float()
                ref = ref.to(dtype)
                assert eng.all_reduce(x)
                torch.cuda.synchronize()
                res["ok"].append(bool(torch.equal(x, ref)))
        # chunked all-reduce (message 3 x the region), reduce-scatter (in place into the
        # bucket's own slice, as ZeRO does) and all-gather (in place), exact on integer data
        n_big = 3 * (16 << 20) // 4 + 1024
        big = torch.arange(n_big, device="cuda", dtype=torch.float32) % 89 + 7.0 * rank
        ref_big = sum(torch.arange(n_big, device="cuda", dtype=torch.float32) % 89 + 7.0 * r for r in range(world))
        assert eng.all_reduce(big)
        torch.cuda.synchronize()
        res["ok"].append(bool(torch.equal(big, ref_big)))
        for ns in (4096, 5 * (16 << 20) // (4 * world) + 512):   # the second needs 3 column bands
            full = torch.arange(world * ns, device="cuda", dtype=torch.float32) % 53 + 3.0 * rank
            want = sum(torch.arange(world * ns, device="cuda", dtype=torch.float32) % 53 + 3.0 * r
                       for r in range(world)).view(world, ns)[rank].clone()
            mine = full.view(world, ns)[rank]
            assert eng.reduce_scatter(mine, full)
            torch.cuda.synchronize()
            res["ok"].append(bool(torch.equal(mine, want)))
            buf = torch.full((world * ns,), -1.0, device="cuda")
            buf.view(world, ns)[rank].copy_(torch.arange(ns, device="cuda", dtype=torch.float32) + 100.0 * rank)
            assert eng.all_gather(buf, buf.view(world, ns)[rank])
            torch.cuda.synchronize()
            want_ag = torch.cat([torch.arange(ns, device="cuda", dtype=torch.float32) + 100.0 * r for r in range(world)])
            res["ok"].append(bool(torch.equal(buf, want_ag)))
        # the auto-mode speed test: every op timed against the (host-side, under gloo) reference,
        # one decision per op shared by both ranks, results recorded for the bench JSON
        t = eng.tune(nbytes=1 << 20, iters=2)
        res["ok"].append(sorted(t) == ["all_gather", "all_reduce", "reduce_scatter"]
                         and all(isinstance(v, bool) for v in eng.use.values()))
        res["error_word"] = eng.error()
        eng.close()
        dist.destroy_process_group()
    except Exception:  # reported by the parent
        res["err"] = traceback.format_exc()
    with open(os.path.join(outdir, f"r{rank}.pkl"), "wb") as f:
        pickle.dump(res, f)


def ulysses_worker(rank, world, nh, nkv, s=32, b=2, d=16):
    """Context-parallel (Ulysses all-to-all) attention on this rank's sequence chunk: returns the
    local output and the local q/k/v gradients for comparison with full-sequence attention."""
    import torch.distributed as dist
    from smdt_amd.parallel import context_parallel as cpar
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        g = torch.Generator().manual_seed(7)
        q = torch.randn(s, b, nh, d, generator=g, dtype=torch.float64)
        k = torch.randn(s, b, nkv, d, generator=g, dtype=torch.float64)
        v = torch.randn(s, b, nkv, d, generator=g, dtype=torch.float64)
        dy = torch.randn(s, b, nh, d, generator=g, dtype=torch.float64)
        ql, kl, vl = (cpar.split_sequence(t).requires_grad_(True) for t in (q, k, v))
        out = cpar.ulysses_attention(ql, kl, vl)
        out.backward(cpar.split_sequence(dy))
        return out.detach(), ql.grad, kl.grad, vl.grad
    finally:
        dist.destroy_process_group()


def gpt_cp_worker(rank, world, tp, cp, sp, cfg_over=None, with_ddp=False):
    """GPT forward/backward with context parallelism (Ulysses) x TP: each CP rank feeds its sequence
    chunk; gradients are averaged over the dp x cp group (by the DDP wrapper when ``with_ddp``).
    Returns the local per-token loss, the full-equivalent gradients and the ranks."""
    import torch.distributed as dist
    from smdt_amd.comm import init_distributed
    from smdt_amd.models.gpt import GPTModel
    from smdt_amd.models.transformer import TransformerConfig
    from smdt_amd.parallel import state as ps
    from smdt_amd.train.utils import context_parallel_slice
    init_distributed("gloo")
    st = ps.initialize_model_parallel(tp, 1, None, cp)
    cfg = TransformerConfig(**{**TINY, **(cfg_over or {}), "sequence_parallel": sp})
    m = GPTModel(cfg)
    tokens, labels = _batch()
    tl, ll = context_parallel_slice(tokens, labels)
    if with_ddp:
        from smdt_amd.parallel.distributed import DistributedDataParallel
        ddp = DistributedDataParallel(m, grad_dtype=torch.float32)
        ddp.zero_grad_buffer()
    loss = m(tl, None, None, labels=ll)
    loss.mean().backward()
    if with_ddp:
        ddp.finish_grad_sync()
        grads = {n: p.main_grad.detach().clone().view_as(p) for n, p in m.named_parameters()}
    else:
        grads = {}
        for n, p in m.named_parameters():
            if p.grad is None:
                continue
            g = p.grad.detach().clone()
            dist.all_reduce(g, group=st.dp_cp_group)
            grads[n] = g / cp
    if sp and tp > 1 and not with_ddp:
        for n, p in m.named_parameters():
            if getattr(p, "sequence_parallel", False) and n in grads:
                dist.all_reduce(grads[n], group=st.tp_group)
    meta = {"tp_rank": st.tp_rank, "cp_rank": st.cp_rank, "layer_offset": m.first_layer,
            "cp_ranks": list(st.cp_ranks), "dp_cp_ranks": list(st.dp_cp_ranks)}
    dist.destroy_process_group()
    return loss.detach(), grads, meta


def gpt_layout_worker(rank, world, tp, pp, nmb, zero, defer=False, sp=False, schedule=None, cfg_over=None,
                      w_fill=False):
    """DDP-wrapped tiny GPT under a TP x PP x DP layout with ``nmb`` micro-batches per step (gradient
    accumulation for pp == 1, 1F1B otherwise): returns the reduced fp32 main_grad of every local
    parameter. The global batch (4 sequences) is split over the DP ranks, so the reduced gradients
    must equal the single-process full-batch gradients (bucket readiness across
    no_sync micro-batches)."""
    import torch.distributed as dist
    from smdt_amd.comm import init_distributed
    from smdt_amd.models.gpt import GPTModel, allreduce_word_embedding_grads
    from smdt_amd.models.transformer import TransformerConfig
    from smdt_amd.parallel import state as ps
    from smdt_amd.parallel.distributed import DistributedDataParallel
    from smdt_amd.train.schedules import get_forward_backward_func, set_pipeline_schedule
    init_distributed("gloo")
    st = ps.initialize_model_parallel(tp, pp)
    if schedule is not None:
        set_pipeline_schedule(schedule)
    if w_fill:
        from smdt_amd.parallel import tensor_parallel as tpm
        tpm.W_FILL = True
    if defer:
        from smdt_amd.parallel import tensor_parallel as tpm
        tpm.DEFERRED_WGRAD.allow_cpu = True
        tpm.DEFERRED_WGRAD.flush_tiles = 2
    cfg = TransformerConfig(**{**TINY, "sequence_parallel": sp, **(cfg_over or {})})
    m = GPTModel(cfg, pre_process=st.is_first_stage(), post_process=st.is_last_stage())
    ddp = DistributedDataParallel(m, bucket_size=6000, use_distributed_optimizer=zero)
    tokens, labels = _batch()
    per = 4 // st.dp
    sl = slice(st.dp_rank * per, (st.dp_rank + 1) * per)
    data = iter(list(zip(tokens[sl].chunk(nmb), labels[sl].chunk(nmb))))

    def fstep(di, model):
        t, lab = next(di)
        o = model(t, None, None, labels=lab)
        return o, (lambda x: (x.mean(), {"loss": x.detach()}))
    ddp.zero_grad_buffer()
    fb = get_forward_backward_func()
    seq = 32 // tp if (sp and tp > 1) else 32
    losses = fb(fstep, data, ddp, nmb, tensor_shape=(seq, per // nmb, 64), dtype=torch.float32)
    ddp.finish_grad_sync()
    allreduce_word_embedding_grads(m)
    full = ddp.grad_data.clone()
    if zero and st.dp > 1:
        for b in ddp.buckets:
            s, e = ddp.shard_range(b)
            dist.all_gather_into_tensor(full[b.start:b.end], ddp.grad_data[s:e].clone(), group=st.dp_group)
    grads = {n: full[ddp.param_index[id(p)][0]:ddp.param_index[id(p)][0] + p.numel()].view_as(p).clone()
             for n, p in m.named_parameters()}
    from smdt_amd.parallel import tensor_parallel as tpm
    meta = {"tp_rank": st.tp_rank, "pp_rank": st.pp_rank, "dp_rank": st.dp_rank, "layer_offset": m.first_layer,
            "wgrad_stats": dict(tpm.DEFERRED_WGRAD.stats)}
    dist.destroy_process_group()
    loss = torch.cat([d["loss"] for d in losses], dim=0) if losses else None   # [b, s] per micro-batch
    return loss, grads, meta


def tp_overlap_order_worker(rank, world):
    """Records the order of ring p2p launches, weight-gradient GEMMs and waits in the backward of
    the sequence-parallel column / row linears, and checks their numerics against plain ops."""
    import torch.distributed as dist
    from smdt_amd.comm import init_distributed
    from smdt_amd.parallel import state as ps
    from smdt_amd.parallel import tensor_parallel as T
    init_distributed("gloo")
    ps.initialize_model_parallel(world, 1)
    T.DEFERRED_WGRAD.allow_cpu = True
    events = []
    real_exchange, real_wgrad = T._exchange, T._wgrad

    class _W:
        def __init__(self, w):
            self.w = w

        def wait(self):
            events.append("wait")
            return self.w.wait()

    def exchange(*a, **k):
        events.append("launch")
        return [_W(w) for w in real_exchange(*a, **k)]

    def wgrad(weight, g2, t2):
        events.append("wgrad")
        return real_wgrad(weight, g2, t2)
    T._exchange, T._wgrad = exchange, wgrad
    g = torch.Generator().manual_seed(5)
    S, B, H, O = 8, 2, 16, 32
    xs = torch.randn(S, B, H, generator=g, dtype=torch.float64)
    w1 = torch.randn(O, H, generator=g, dtype=torch.float64)     # column: full weight (rank shard below)
    b1 = torch.randn(O, generator=g, dtype=torch.float64)
    w2 = torch.randn(H, O, generator=g, dtype=torch.float64)     # row
    dy = torch.randn(S, B, H, generator=g, dtype=torch.float64)
    n = S // world
    o = O // world
    wc = torch.nn.Parameter(w1[rank * o:(rank + 1) * o].clone())
    bc = torch.nn.Parameter(b1[rank * o:(rank + 1) * o].clone())
    wr = torch.nn.Parameter(w2[:, rank * o:(rank + 1) * o].clone())
    for p in (wc, bc, wr):
        p.main_grad = torch.zeros_like(p)
        p._smdt_grad_ready = lambda _p: None
    x = xs[rank * n:(rank + 1) * n].clone().requires_grad_(True)
    h = T.column_sp_linear(x, wc, bc)
    y = T.row_sp_linear(h, wr)
    events.append("backward")
    y.backward(dy[rank * n:(rank + 1) * n])
    T.DEFERRED_WGRAD.flush()
    # reference on the full problem
    xr = xs.clone().requires_grad_(True)
    w1r, b1r, w2r = (t.clone().requires_grad_(True) for t in (w1, b1, w2))
    yr = torch.nn.functional.linear(torch.nn.functional.linear(xr, w1r, b1r), w2r)
    yr.backward(dy)
    torch.testing.assert_close(y.detach(), yr.detach()[rank * n:(rank + 1) * n])
    torch.testing.assert_close(x.grad, xr.grad[rank * n:(rank + 1) * n])
    torch.testing.assert_close(wc.main_grad, w1r.grad[rank * o:(rank + 1) * o])
    bgrad = bc.main_grad + (bc.grad if bc.grad is not None else 0)   # CPU: returned to autograd
    torch.testing.assert_close(bgrad, b1r.grad[rank * o:(rank + 1) * o])
    torch.testing.assert_close(wr.main_grad, w2r.grad[:, rank * o:(rank + 1) * o])
    dist.destroy_process_group()
    return events


def saved_bytes_worker(rank, world, tp, cfg_over):
    """TP run of the tiny GPT with ``cfg_over`` (recompute settings): returns (loss, grads, meta,
    bytes of tensors autograd saved during forward)."""
    import torch.distributed as dist
    from smdt_amd.comm import init_distributed
    from smdt_amd.models.gpt import GPTModel
    from smdt_amd.models.transformer import TransformerConfig
    from smdt_amd.parallel import state as ps
    init_distributed("gloo")
    st = ps.initialize_model_parallel(tp, 1)
    cfg = TransformerConfig(**{**TINY, **cfg_over})
    m = GPTModel(cfg)
    tokens, labels = _batch()
    seen = {}

    def pack(t):
        seen[id(t)] = t.numel() * t.element_size() if t.layout == torch.strided else 0
        return t
    with torch.autograd.graph.saved_tensors_hooks(pack, lambda t: t):
        loss = m(tokens, None, None, labels=labels)
    loss.mean().backward()
    grads = {n: p.grad.detach().clone() for n, p in m.named_parameters() if p.grad is not None}
    meta = {"tp_rank": st.tp_rank, "pp_rank": 0, "layer_offset": 0}
    if dist.is_initialized():
        dist.destroy_process_group()
    return loss.detach(), grads, meta, sum(seen.values())


def relay_ipc_worker(rank, world, port, outdir):
    """One rank of the cross-process relay test: 4 processes on cuda:0, TP pairs (0,1) and (2,3),
    gloo carrying the IPC handles and the reference p2p; the exchanges themselves are the kernel."""
    import os
    import pickle
    import traceback

    import torch

    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "RANK": str(rank),
                       "WORLD_SIZE": str(world)})
    res = {"ok": [], "err": None, "error_word": None}
    try:
        import torch.distributed as dist
        from smdt_amd.comm import relay
        from smdt_amd.parallel import tensor_parallel as tpl
        dist.init_process_group("gloo", rank=rank, world_size=world)
        torch.cuda.set_device(0)
        groups = [dist.new_group([0, 1]), dist.new_group([2, 3])]
        pg = groups[rank // 2]
        partner = rank ^ 1
        eng = relay.XgmiRelay(pg, slot_bytes=1 << 20, sub=2, validate=True)  # checked against p2p
        res["ok"].append(eng.active)
        # the run-time speed test runs and reaches one decision on every rank (timings through
        # gloo's host copies are meaningless here; the decision logic is what is exercised)
        t = eng.tune(sizes=(64 << 10, 256 << 10), iters=2)
        res["ok"].append(sorted(t) == [64 << 10, 256 << 10] and eng.active == (eng.min_bytes is not None))
        eng.active, eng.min_bytes = True, 0
        subs = eng.tune_sub(nbytes=1 << 20, iters=2)     # one decision on every rank
        res["ok"].append(sorted(subs) == [1, 2, 4] and eng.sub in (1, 2, 4) and eng.cu_blocks() == 2 * world * eng.sub)
        # a message of 3 calls (fp32) and a short bf16 one
        for n, dt in ((3 * world * (1 << 20) // 2 // 4 + 400, torch.float32), (777 * 8, torch.bfloat16)):
            base = torch.arange(n, device="cuda", dtype=torch.float32) % 113
            x = (base + 10.0 * rank).to(dt)
            y = torch.empty_like(x)
            assert eng.exchange(x, y)
            torch.cuda.synchronize()
            res["ok"].append(bool(torch.equal(y, (base + 10.0 * partner).to(dt))))
        x = torch.full((4096,), float(rank), device="cuda")
        y = torch.empty_like(x)
        h = eng.exchange_async(x, y)
        h.wait()
        torch.cuda.synchronize()
        res["ok"].append(bool((y == partner).all()))
        # the tensor-parallel ring steps routed through the relay
        relay._ENGINES[id(pg)] = eng
        me = dist.get_rank(pg)
        for dt in (torch.float32, torch.bfloat16):
            mk = lambda r: (torch.arange(8 * 16, device="cuda", dtype=torch.float32).view(8, 16) + 100.0 * r).to(dt)
            total = tpl.ag_ring(mk(rank), pg)
            parts = [mk(rank), mk(partner)] if me == 0 else [mk(partner), mk(rank)]
            torch.cuda.synchronize()
            res["ok"].append(bool(torch.equal(total, torch.cat(parts))))
            full = lambda r: (torch.arange(16 * 16, device="cuda", dtype=torch.float32).view(16, 16) % 7 * (r + 1)).to(dt)
            got = tpl.rs_ring(lambda lo, m, o: full(rank)[lo:lo + m].clone(), pg, (16, 16), full(rank))
            exp = (full(rank).float() + full(partner).float())[me * 8:(me + 1) * 8].to(dt)
            torch.cuda.synchronize()
            res["ok"].append(bool(torch.equal(got, exp)))
        del relay._ENGINES[id(pg)]
        res["error_word"] = eng.error()
        eng.close()
        dist.destroy_process_group()
    except Exception:
        res["err"] = traceback.format_exc()
    with open(os.path.join(outdir, f"r{rank}.pkl"), "wb") as f:
        pickle.dump(res, f)


def relay_tp_mlp_worker(rank, world, port, outdir):
    """One rank of the relay-backed tensor-parallel MLP test: 4 processes on cuda:0, TP pairs
    (0,1) (2,3) with sequence parallelism; every TP ring exchange (forward all-gather /
    reduce-scatter, backward reduce-scatter / all-gather) goes through the xGMI relay kernel over
    HIP-IPC mappings. Each rank checks its output / gradient shards against an fp32 reference of
    the full MLP computed in-process."""
    import os
    import pickle
    import traceback

    import torch

    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "RANK": str(rank),
                       "WORLD_SIZE": str(world)})
    res = {"err": None, "rel": {}, "calls": 0, "error_word": None}
    try:
        import torch.distributed as dist
        import torch.nn.functional as F
        from smdt_amd.comm import relay
        from smdt_amd.parallel import state as ps
        from smdt_amd.parallel import tensor_parallel as tpl
        dist.init_process_group("gloo", rank=rank, world_size=world)
        torch.cuda.set_device(0)
        st = ps.initialize_model_parallel(2)
        eng = relay.XgmiRelay(st.tp_group, slot_bytes=1 << 20, sub=2)
        relay._ENGINES[id(st.tp_group)] = eng
        h, ffn, s, b = 256, 1024, 128, 4
        dev = torch.device("cuda", 0)
        fc1 = tpl.ColumnParallelLinear(h, ffn, bias=True, key="fc1", params_dtype=torch.bfloat16, device=dev,
                                       sequence_parallel=True)
        fc2 = tpl.RowParallelLinear(ffn, h, bias=False, key="fc2", params_dtype=torch.bfloat16, device=dev,
                                    sequence_parallel=True)
        with torch.no_grad():
            fc1.bias.copy_(torch.linspace(-0.5, 0.5, ffn, device=dev)[st.tp_rank * (ffn // 2):][: ffn // 2])
        w1 = tpl.init_full_then_shard((ffn, h), 0.02, "fc1.weight", 1234, torch.float32, dev, None, 0, 1)
        w2 = tpl.init_full_then_shard((h, ffn), 0.02, "fc2.weight", 1234, torch.float32, dev, None, 0, 1)
        w1 = w1.to(torch.bfloat16).float().requires_grad_(True)
        w2 = w2.to(torch.bfloat16).float().requires_grad_(True)
        b1 = torch.linspace(-0.5, 0.5, ffn, device=dev).to(torch.bfloat16).float().requires_grad_(True)
        g = torch.Generator(device=dev)
        g.manual_seed(100 + rank // 2)  # one input per TP pair
        x_full = torch.randn(s, b, h, device=dev, generator=g).to(torch.bfloat16)
        gy_full = torch.randn(s, b, h, device=dev, generator=g)
        lo, hi = st.tp_rank * (s // 2), (st.tp_rank + 1) * (s // 2)
        for it in range(2):  # two iterations: both slot parities and the freed-slot handshake
            x = x_full[lo:hi].clone().requires_grad_(True)
            y = fc2(F.gelu(fc1(x), approximate="tanh"))
            (y.float() * gy_full[lo:hi]).sum().backward()
            tpl.DEFERRED_WGRAD.flush()
            torch.cuda.synchronize()
            xr = x_full.float().requires_grad_(True)
            for t in (w1, w2, b1):
                t.grad = None
            yr = F.linear(F.gelu(F.linear(xr, w1, b1), approximate="tanh"), w2)
            (yr * gy_full).sum().backward()

            def rel(a, r):
                return float((a.float() - r).norm() / (r.norm() + 1e-12))
            f0, f1 = st.tp_rank * (ffn // 2), (st.tp_rank + 1) * (ffn // 2)
            res["rel"][f"y{it}"] = rel(y, yr[lo:hi].detach())
            res["rel"][f"dx{it}"] = rel(x.grad, xr.grad[lo:hi])
            res["rel"][f"dw1_{it}"] = rel(fc1.weight.grad, w1.grad[f0:f1])
            res["rel"][f"db1_{it}"] = rel(fc1.bias.grad, b1.grad[f0:f1])
            res["rel"][f"dw2_{it}"] = rel(fc2.weight.grad, w2.grad[:, f0:f1])
            for p in (fc1.weight, fc1.bias, fc2.weight):
                p.grad = None
        res["calls"] = eng.calls
        res["error_word"] = eng.error()
        del relay._ENGINES[id(st.tp_group)]
        eng.close()
        dist.destroy_process_group()
    except Exception:
        res["err"] = traceback.format_exc()
    with open(os.path.join(outdir, f"r{rank}.pkl"), "wb") as f:
        pickle.dump(res, f)


def cp_rng_resume_worker(rank, world, save_dir, async_save=False):
    """cp = 2: save a checkpoint, keep drawing dropout masks, reload, draw again. Each CP rank must
    resume ITS OWN Philox streams (they are shifted per cp_rank), not cp_rank 0's."""
    import torch.distributed as dist
    from smdt_amd.comm import init_distributed
    from smdt_amd.models.gpt import GPTModel
    from smdt_amd.models.transformer import TransformerConfig
    from smdt_amd.parallel import state as ps
    from smdt_amd.parallel.random import get_rng, model_parallel_seed
    from smdt_amd.train.checkpointing import finalize_async_save, load_checkpoint, save_checkpoint
    init_distributed("gloo")
    st = ps.initialize_model_parallel(1, 1, None, 2)
    model_parallel_seed(1234)
    m = GPTModel(TransformerConfig(**TINY))

    def mask():   # the fused dropout kernels' masks are a pure function of (seed, offset)
        return (get_rng("default").next(), get_rng("tp").next(), float(torch.rand(1)))
    mask()                                   # advance the streams a little before saving
    save_checkpoint(3, m, save_dir=save_dir, async_save=async_save)
    after_save = [mask(), mask()]
    assert finalize_async_save(blocking=True)   # (no-op for a synchronous save)
    model_parallel_seed(99)                  # a fresh process would start elsewhere
    load_checkpoint(m, load_dir=save_dir)
    resumed = [mask(), mask()]
    out = {"cp_rank": st.cp_rank, "same": after_save == resumed, "mask": after_save[0]}
    dist.destroy_process_group()
    return out


class _FakeXgmi:
    """Stand-in for comm/xgmi.XgmiAllReduce on gloo: the same call protocol, with a timeout that
    can be injected — from call ``trip_at`` on, this rank's outputs are NaN-filled and its sticky
    error word is set, exactly what the kernel does when a peer never arrives."""

    class _H:
        def wait(self):
            return True

        def timing(self):
            return None

    def __init__(self, group, trip_at=None):
        import torch.distributed as dist
        self.group, self.trip_at, self.calls, self.active = group, trip_at, 0, True
        self.ws = dist.get_world_size(group)
        self.err = torch.zeros(1, dtype=torch.int32)

    def error_tensor(self):
        return self.err

    def deactivate(self, reason=""):
        self.active = False

    def _after(self, out):
        self.calls += 1
        if self.trip_at is not None and self.calls >= self.trip_at:
            self.err.fill_(1)
        if int(self.err[0]):
            out.fill_(float("nan"))
        return self._H()

    def reduce_scatter_async(self, out, inp, op="sum"):
        import torch.distributed as dist
        if not self.active:
            return None
        dist.reduce_scatter_tensor(out, inp, group=self.group)
        if op == "avg":
            out.div_(self.ws)
        return self._after(out)

    def all_gather_async(self, out, inp):
        import torch.distributed as dist
        if not self.active:
            return None
        dist.all_gather_into_tensor(out, inp.clone(), group=self.group)
        return self._after(out)

    def all_reduce_async(self, t, op="sum"):
        import torch.distributed as dist
        if not self.active:
            return None
        dist.all_reduce(t, group=self.group)
        if op == "avg":
            t.div_(self.ws)
        return self._after(t)


def xgmi_fallback_worker(rank, world, trip_rank, trip_step, steps=6):
    """DDP + ZeRO-1 + MixedPrecisionAdam on an engine that times out on ``trip_rank`` in the first
    gradient reduce-scatter of step ``trip_step`` (1-based): the health monitor must switch every rank to the default transport at the same
    step, warn once, repair the gathered parameters, and keep every loss finite."""
    import math
    import warnings
    import torch.distributed as dist
    from smdt_amd.comm import health
    from smdt_amd.optim.optimizer import MixedPrecisionAdam
    from smdt_amd.parallel import state as ps
    from smdt_amd.parallel.distributed import DistributedDataParallel
    dist.init_process_group("gloo")
    ps.initialize_model_parallel(1, 1)
    health.reset()
    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Linear(32, 64), torch.nn.GELU(), torch.nn.Linear(64, 32))
    ddp = DistributedDataParallel(model, bucket_size=1024, use_distributed_optimizer=True)
    per_step = 2 * len(ddp.buckets)                   # one reduce-scatter + one all-gather per bucket
    eng = _FakeXgmi(ddp.dp_group, (trip_step - 1) * per_step + 1 if rank == trip_rank else None)
    ddp.xgmi = eng
    health.register(eng)
    opt = MixedPrecisionAdam(ddp, lr=1e-2, weight_decay=0.0, clip_grad=1.0)
    gen = torch.Generator().manual_seed(100 + rank)
    losses, active = [], []
    with warnings.catch_warnings(record=True) as caught:
        warnings.simplefilter("always")
        for _ in range(steps):
            ddp.zero_grad_buffer()
            x = torch.randn(8, 32, generator=gen)
            loss = (ddp(x) - x).pow(2).mean()
            loss.backward()
            ddp.finish_grad_sync()
            opt.step()
            losses.append(float(loss))
            active.append(eng.active)
    params = torch.cat([p.detach().flatten() for p in model.parameters()])
    gathered = [torch.empty_like(params) for _ in range(world)]
    dist.all_gather(gathered, params)
    out = {"losses": losses, "active": active, "events": list(health.EVENTS),
           "warned": any("timed-out peer" in str(w.message) for w in caught),
           "finite": all(math.isfinite(v) for v in losses) and bool(torch.isfinite(params).all()),
           "replicas_equal": all(torch.equal(gathered[0], g) for g in gathered)}
    dist.destroy_process_group()
    return out


def xgmi_timeout_worker(rank, world, port, outdir):
    """Real kernel, real IPC (both ranks on cuda:0, gloo carries the handles): rank 0's spin limit is
    lowered and rank 1 arrives late, so rank 0's call times out — its sticky error word is set
    (read through the aliasing device tensor), its output is NaN-filled, and the health monitor
    switches BOTH ranks' engines off at the same step."""
    import os
    import pickle
    import time
    import traceback

    import torch
    from smdt_amd.comm import health, xgmi

    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "RANK": str(rank),
                       "WORLD_SIZE": str(world)})
    res = {"err": None}
    try:
        import torch.distributed as dist
        dist.init_process_group("gloo", rank=rank, world_size=world)
        torch.cuda.set_device(0)
        health.reset()
        eng = xgmi.XgmiAllReduce(None, region_bytes=4 << 20, blocks=8, validate=False)
        x = torch.ones(4096, device="cuda")
        assert eng.all_reduce(x)                      # a healthy call first
        torch.cuda.synchronize()
        res["first_ok"] = bool(torch.equal(x, torch.full_like(x, float(world))))
        if rank == 0:
            eng.set_spin_limit(2000)                  # ~ms instead of ~seconds
        dist.barrier()
        if rank == 1:
            time.sleep(1.0)                           # arrive long after rank 0 gave up
        y = torch.ones(4096, device="cuda")
        eng.all_reduce(y)
        torch.cuda.synchronize()
        res["nan_out"] = bool(torch.isnan(y).all())
        res["error_word"] = int(eng.error_tensor().item())
        mon = health.monitor()
        mon.launch()                                  # end of "step k": agree on the flag
        mon.consume()                                 # start of "step k + 1": fall back
        res["active_after"] = eng.active
        res["events"] = list(health.EVENTS)
        eng.close()
        dist.destroy_process_group()
    except Exception:  # reported by the parent
        res["err"] = traceback.format_exc()
    with open(os.path.join(outdir, f"r{rank}.pkl"), "wb") as f:
        pickle.dump(res, f)


def smddp_torch_ddp_worker(rank, world, port, outdir):
    """One rank of the smddp-backend GPU test: unmodified torch DDP on the ``smddp`` group, every
    rank on cuda:0 (Gloo underneath, SMDT_SMDDP_INNER=gloo), bucket all-reduces through the xGMI
    engine of comm/smddp.SMDDPProcessGroup; gradients vs the mean of per-rank local gradients."""
    import os
    import pickle
    import traceback

    import torch
    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "RANK": str(rank),
                       "WORLD_SIZE": str(world), "SMDT_SMDDP_INNER": "gloo"})
    res = {"err": None}
    try:
        import torch.distributed as dist
        import smdt_amd.comm.smddp as S
        torch.cuda.set_device(0)
        dist.init_process_group("smddp", rank=rank, world_size=world)
        torch.manual_seed(0)
        def mlp():
            return torch.nn.Sequential(torch.nn.Linear(64, 256), torch.nn.GELU(), torch.nn.Linear(256, 256),
                                       torch.nn.GELU(), torch.nn.Linear(256, 256), torch.nn.GELU(),
                                       torch.nn.Linear(256, 32)).cuda()
        m = mlp()
        ref_m = mlp()
        ref_m.load_state_dict(m.state_dict())
        # torch 2.10's DDP keeps ONE bucket for a model this size (bucket_cap_mb splits only with
        # find_unused_parameters, whose unused-parameter scan syncs the host itself): one bucket
        # all-reduce per backward, launched from the autograd hook before backward returns
        ddp = torch.nn.parallel.DistributedDataParallel(m)
        mod = m
        from smdt_amd.comm import stats as cstats
        ok, placement = [], []
        for step in range(5):
            x = torch.randn(16, 64, generator=torch.Generator().manual_seed(10 * step + rank)).cuda()
            mod.zero_grad()
            measured = step >= 3      # steady state (bucket rebuild and the engine build are over)
            if measured:
                torch.cuda.synchronize()
                cstats.enable(True)
                cstats.begin_step()      # engine calls record start events inside a stats step
                S._TIMINGS.clear()
                torch.cuda.set_sync_debug_mode("error")   # any host sync in the hook path raises
                b0 = torch.cuda.Event(enable_timing=True)
                b1 = torch.cuda.Event(enable_timing=True)
                b0.record()
            ddp(x).square().mean().backward()
            if measured:
                b1.record()
                torch.cuda.set_sync_debug_mode(0)
                cstats.end_step()
                cstats.enable(False)
                torch.cuda.synchronize()
                pg = dist.distributed_c10d._get_default_group()
                starts = [b0.elapsed_time(a) for a, _ in S._TIMINGS]
                placement.append({"n": len(S._TIMINGS), "engine_stream": pg._engine._stream != torch.cuda.current_stream(),
                                  "first_start_ms": min(starts) if starts else None,
                                  "backward_ms": b0.elapsed_time(b1)})
            ref_m.zero_grad()
            ref_m(x).square().mean().backward()
            for p, q in zip(mod.parameters(), ref_m.parameters()):
                mean = q.grad.cpu()
                dist.all_reduce(mean)            # a CPU tensor: the Gloo path of the smddp group
                ok.append(bool(torch.allclose(p.grad.cpu(), mean / world, atol=1e-5, rtol=1e-4)))
        torch.cuda.synchronize()
        pg = dist.distributed_c10d._get_default_group()   # the SMDDPProcessGroup itself
        res.update(ok=ok, stats=S.smddp_stats(), backend=dist.get_backend(), placement=placement,
                   error_word=pg._engine.error() if getattr(pg, "_engine", None) is not None else None)
        dist.barrier()
        dist.destroy_process_group()
    except Exception:  # noqa: BLE001
        res["err"] = traceback.format_exc()
    with open(os.path.join(outdir, f"r{rank}.pkl"), "wb") as f:
        pickle.dump(res, f)


def tp_direct_worker(rank, world, port, outdir):
    """One rank of the direct-TP-exchange GPU test: ``world`` processes on cuda:0 with a Gloo
    world group, the TP group's xGMI engine over same-device IPC (comm/tp_direct.TpDirect.for_test),
    and the sequence-parallel ring entry points ``ag_ring`` / ``rs_ring`` run through it; results vs
    the host-side gathered / reduced reference."""
    import os
    import pickle
    import traceback

    import torch
    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "RANK": str(rank),
                       "WORLD_SIZE": str(world), "HSA_ENABLE_IPC_MODE_LEGACY": "0"})
    res = {"err": None}
    try:
        import torch.distributed as dist
        from smdt_amd.comm import tp_direct
        from smdt_amd.parallel import state as ps
        from smdt_amd.parallel import tensor_parallel as T
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        st = ps.initialize_model_parallel(world, 1)
        st.tp_direct = tp_direct.TpDirect.for_test(st.tp_group)
        g = st.tp_group
        torch.manual_seed(100 + rank)
        n, h, o = 256, 64, 96
        x = torch.randn(n, 4, h, device="cuda", dtype=torch.bfloat16)
        w = torch.randn(o, h, device="cuda", dtype=torch.bfloat16)
        xs = [torch.empty_like(x.cpu()) for _ in range(world)]
        dist.all_gather(xs, x.cpu())
        ref_total = torch.cat(xs)
        full = torch.randn(n * world, 4, o, device="cuda", dtype=torch.float32)
        fulls = [torch.empty_like(full.cpu()) for _ in range(world)]
        dist.all_gather(fulls, full.cpu())
        red = fulls[0].clone()
        for t in fulls[1:]:       # rank order, fp32: the engine's summation order
            red += t
        oks = {}
        for k in (1, 2, 4):   # row pieces per exchange (1 = whole chunks)
            tp_direct.PIECES = k
            # all-gather with a per-row-range GEMM (the column-parallel forward)
            out = torch.empty(n * world, 4, o, device="cuda", dtype=torch.bfloat16)
            seen = []

            def chunk(lo, ch):
                seen.append((lo, ch.shape[0]))
                out[lo:lo + ch.shape[0]].copy_(ch @ w.t())
            total = T.ag_ring(x, g, chunk)
            cover = sorted(seen)
            ok_ag = (torch.equal(total.cpu(), ref_total) and seen[0] == (rank * n, n)
                     and sum(m for _, m in seen) == n * world
                     and all(a + m == b for (a, m), (b, _) in zip(cover, cover[1:]))
                     and len(seen) == 1 + ((world - 1) * k if k > 1 else (1 if rank in (0, world - 1) else 2)))
            ok_mm = torch.allclose(out.float().cpu(), (ref_total.float() @ w.float().cpu().t()), atol=0.5, rtol=2e-2)
            # reduce-scatter of per-row-range partials (the row-parallel forward), bit-exact: the
            # engine sums in rank order in fp32, as the host reference below does
            calls = []

            def part(lo, m, dst):
                calls.append((lo, m))
                src = full[lo:lo + m] * 1.0
                if dst is None:
                    return src
                dst.copy_(src)
                return dst
            got = T.rs_ring(part, g, full.shape, full, before_last_wait=lambda: seen.append("wgrad"))
            ok_rs = torch.equal(got.cpu(), red[rank * n:(rank + 1) * n]) and len(calls) == (world * k if k > 1 else 1)
            oks[k] = (bool(ok_ag), bool(ok_mm), bool(ok_rs), "wgrad" in seen)
        tp_direct.PIECES = 2
        ok_ag = all(v[0] for v in oks.values())
        ok_mm = all(v[1] for v in oks.values())
        ok_rs = all(v[2] for v in oks.values())
        res["pieces"] = oks
        res["pieces_issued"] = st.tp_direct.pieces_issued
        torch.cuda.synchronize()
        res.update(ok_ag=bool(ok_ag), ok_mm=bool(ok_mm), ok_rs=bool(ok_rs), calls=st.tp_direct.calls,
                   wgrad_hook=all(v[3] for v in oks.values()), error_word=st.tp_direct.eng.error())
        dist.barrier()
        st.tp_direct.eng.close()
        dist.destroy_process_group()
    except Exception:  # noqa: BLE001
        res["err"] = traceback.format_exc()
    with open(os.path.join(outdir, f"r{rank}.pkl"), "wb") as f:
        pickle.dump(res, f)


def sp_gather_slots_worker():
    """(one GPU process) A TP2 + SP GPT rank emulated on a loopback group: forward + backward with
    the sequence-parallel norms writing into their all-gather slots (no local copy in ag_ring),
    then again with the slots off. Prints one JSON line: max |diff| of the loss and of every
    gradient, and the ag_ring in-place / copied counts of each pass."""
    import json
    from smdt_amd.models.gpt import GPTModel
    from smdt_amd.models.transformer import TransformerConfig
    from smdt_amd.parallel import state as ps
    from smdt_amd.parallel import tensor_parallel as tp
    from smdt_amd.parallel.random import model_parallel_seed
    ps.initialize_emulated_tensor_parallel(2)
    model_parallel_seed(1234)
    cfg = TransformerConfig(num_layers=2, hidden_size=256, num_attention_heads=4, max_position_embeddings=128,
                            padded_vocab_size=512, hidden_dropout=0.0, attention_dropout=0.0,
                            params_dtype=torch.bfloat16, sequence_parallel=True, use_flash_attn=True)
    model = GPTModel(cfg, device="cuda")
    g = torch.Generator(device="cuda")
    g.manual_seed(7)
    toks = torch.randint(0, 500, (4, 129), device="cuda", generator=g)

    def run():
        for p in model.parameters():
            p.grad = None
        tp.AG_RING_STATS.update(in_place=0, copied=0)
        loss = model(toks[:, :-1], None, None, labels=toks[:, 1:]).float().mean()
        loss.backward()
        torch.cuda.synchronize()
        return loss.detach(), {n: p.grad.float().clone() for n, p in model.named_parameters() if p.grad is not None}, \
            dict(tp.AG_RING_STATS)
    l1, g1, s1 = run()
    orig = tp.sp_gather_spec
    tp.sp_gather_spec = lambda: None
    try:
        l0, g0, s0 = run()
    finally:
        tp.sp_gather_spec = orig
    diff = max(float((g1[k] - g0[k]).abs().max()) for k in g0)
    print(json.dumps({"loss_diff": float((l1 - l0).abs()), "grad_max_diff": diff, "n_grads": len(g0),
                      "same_keys": sorted(g0) == sorted(g1), "stats_slots": s1, "stats_copy": s0}), flush=True)


def sft_window_agreement_worker(rank, world, tmpdir, ds_cfg, nofit_rank, fuse_ga):
    """The SFT Trainer on ``world`` Gloo ranks for 2 optimizer steps (GA 2) where only rank
    ``nofit_rank`` finds its fused accumulation window too large (``Trainer._window_fits``
    False there, True elsewhere). The decision must be agreed across the data-parallel group:
    otherwise the ranks issue different numbers of ZeRO collectives and hang or mis-reduce.
    Returns (full parameters, (fused, unfused) window counts logged by the trainer)."""
    from smdt_amd.models.hf import HFCausalLM
    from smdt_amd.data import sft
    from smdt_amd.parallel import state as ps
    from smdt_amd.train import hf_args
    from smdt_amd.train.sft_trainer import Trainer
    os.environ["SMDT_SFT_FUSE_GA"] = "1" if fuse_ga else "0"
    # the two runs are compared bit-exactly: one intra-op thread, so the CPU GEMMs' reduction
    # split cannot follow the machine's load (a parallel test run flipped bf16 ulps otherwise)
    torch.set_num_threads(1)
    Trainer._window_fits = lambda self, window: self.rank != nofit_rank
    ps.destroy_model_parallel()
    torch.manual_seed(0)
    model = HFCausalLM(SFT_LLAMA, params_dtype=torch.float32)
    tok = sft.HashWordTokenizer(120, 48, pad_token="<pad>", special_ids={"<pad>": 0, "</s>": 1, "<s>": 2, "<unk>": 3})
    path = os.path.join(tmpdir, "alpaca.json")
    if rank == 0 and not os.path.exists(path):
        sft.write_synthetic_alpaca(path + ".tmp", 40, seed=1)
        os.replace(path + ".tmp", path)
    while not os.path.exists(path):
        time.sleep(0.05)
    ds = sft.SupervisedDataset(path, tok)
    p = hf_args.ArgumentParser((hf_args.ModelArguments, hf_args.DataArguments, hf_args.TrainingArguments))
    argv = ["--output_dir", os.path.join(tmpdir, f"out{int(fuse_ga)}{nofit_rank}"), "--per_device_train_batch_size", "2",
            "--gradient_accumulation_steps", "2", "--learning_rate", "1e-3", "--logging_steps", "1",
            "--save_steps", "0", "--max_steps", "2", "--deepspeed", ds_cfg, "--pad_to_multiple_of", "8",
            "--warmup_steps", "1", "--seed", "5"]
    args = p.parse_args_into_dataclasses(argv)[2]
    logs = []
    t = Trainer(model=model, tokenizer=tok, args=args, train_dataset=ds,
                data_collator=sft.DataCollatorForSupervisedDataset(tok, 8))
    t._log0 = lambda msg: logs.append(msg)
    t.train()
    with t.engine.gathered_params():
        full = {k: v.detach().clone() for k, v in t.model.named_parameters()}
    return full, [m for m in logs if "[sft]" in m]


def deterministic_fold_worker(rank, world, zero):
    """DistributedDataParallel(deterministic_reduce=True): each rank's gradient buffer holds
    rank-seeded values; returns the reduced buffer (this rank's shard region for ZeRO-1)."""
    import torch.distributed as dist
    from smdt_amd.comm import init_distributed
    from smdt_amd.parallel import state as ps
    from smdt_amd.parallel.distributed import DistributedDataParallel
    init_distributed("gloo")
    ps.initialize_model_parallel(1, 1)
    m = torch.nn.Sequential(torch.nn.Linear(64, 96), torch.nn.Linear(96, 48))
    ddp = DistributedDataParallel(m, bucket_size=3000, use_distributed_optimizer=zero, deterministic_reduce=True)
    ddp.zero_grad_buffer()
    g = torch.Generator().manual_seed(100 + rank)
    ddp.grad_data.copy_(torch.randn(ddp.grad_data.numel(), generator=g) * torch.logspace(-6, 3, ddp.grad_data.numel()))
    for b in ddp.buckets:
        ddp._launch(b)
    ddp.finish_grad_sync()
    ranges = [ddp.shard_range(b) for b in ddp.buckets] if zero else [(0, ddp.grad_data.numel())]
    out = (ddp.grad_data.clone(), ranges)
    dist.destroy_process_group()
    return out


def ag_start_view_worker(rank, world, emulate=False):
    """``tp.ag_start`` on the first output of a multi-output autograd node that is a VIEW of the
    all-gather buffer (what the fused sequence-parallel norm returns on the GPU), then the column
    SP linear over it and its backward: the receive into the buffer must stay invisible to
    autograd (it goes through ``.data``). Returns (out, dx) for comparison with the plain ring."""
    import torch.distributed as dist
    from smdt_amd.comm import init_distributed
    from smdt_amd.parallel import state as ps
    from smdt_amd.parallel import tensor_parallel as TPm
    init_distributed("gloo")
    if emulate:   # one process as TP rank 0 of 2: the exchange is an in-place local copy
        st = ps.initialize_emulated_tensor_parallel(2, 1)
    else:
        st = ps.initialize_model_parallel(2, 1)
    rank = st.tp_rank
    torch.manual_seed(0)
    n, b, h, o = 4, 2, 8, 6
    full_x = torch.randn(2 * n, b, h)
    w = torch.randn(o, h, requires_grad=True)

    class _Producer(torch.autograd.Function):
        """Writes 2x its input into its slot of a fresh gather buffer; returns (view, other)."""
        @staticmethod
        def forward(ctx, x):
            buf = x.new_empty((2 * n, b, h))
            buf[rank * n:(rank + 1) * n].copy_(2 * x)
            y = buf[rank * n:(rank + 1) * n]
            y._smdt_gather = (buf, rank)
            return y, x * 3

        @staticmethod
        def backward(ctx, gy, gs):
            return 2 * gy + 3 * gs

    res = {}
    for mode in ("ring", "started"):
        x = full_x[rank * n:(rank + 1) * n].clone().requires_grad_(True)
        y, s = _Producer.apply(x)
        if mode == "started":
            TPm.ag_start(y, st.tp_group)
        out = TPm._ColumnSPLinear.apply(y, w, None)
        (out.sum() + s.sum()).backward()
        res[mode] = (out.detach().clone(), x.grad.detach().clone())
        w.grad = None
    dist.destroy_process_group()
    return res


def deferred_add_worker(rank, world, case, guard=True, defer=True, pending_guard=True):
    """tp2 + SP on Gloo with the ring reduce-scatter's combine deferred to the consuming fused norm
    (tensor_parallel.defer_rs_add). ``case``:
      * "hook": a forward hook on layer 0's attention output projection (a row-parallel linear)
        records its output; ``guard`` False disables the foreign-hook check (mutation arm);
      * "plain_norm": the layers' norm replaced by a plain one that never takes the pending summand;
      * "bwd": the column-parallel linears' backward reduce-scatter is made to defer its combine
        (forced on CPU), and the norm backward on CPU does not take it.
    ``pending_guard`` False turns the forward guard off (``PendingPartial``: any read of a pending
    row-parallel output other than its fused norm's raises).
    Returns (loss or the raised error text, hook capture, split stats)."""
    import torch.nn.functional as F
    import torch.distributed as dist
    from smdt_amd.comm import init_distributed
    from smdt_amd.models import transformer as T
    from smdt_amd.models.gpt import GPTModel
    from smdt_amd.models.transformer import TransformerConfig
    from smdt_amd.parallel import state as ps
    from smdt_amd.parallel import tensor_parallel as TPm
    init_distributed("gloo")
    ps.initialize_model_parallel(2, 1)
    TPm._DEFER_RS_ADD = defer
    TPm._GUARD = pending_guard
    for k in TPm.SPLIT_STATS:
        TPm.SPLIT_STATS[k] = 0
    if not guard:
        TPm.foreign_hooks = lambda module: False
    if case == "plain_norm":
        def plain(self, x, xbias, residual, p, training, gather=None):
            h = x if xbias is None else x + xbias
            s = h if residual is None else residual + h
            return F.layer_norm(s, s.shape[-1:], self.weight, self.bias, self.eps), s
        T.Norm.fused = plain
    if case == "bwd":
        TPm._bwd_add_to_norm = lambda x: True
    if case == "second_consumer":
        fused = T.Norm.fused

        def twice(self, x, *a, **k):
            _ = x.float().abs().max()          # a second reader of the row-parallel output
            return fused(self, x, *a, **k)
        T.Norm.fused = twice
    cfg = TransformerConfig(**{**TINY, "sequence_parallel": True})
    m = GPTModel(cfg)
    seen = []
    if case == "hook":
        m.decoder.layers[0].attention.proj.register_forward_hook(
            lambda mod, inp, out: seen.append((out[0] if isinstance(out, tuple) else out).detach().clone()))
    tokens, labels = _batch()
    try:
        loss = m(tokens, None, None, labels=labels)
        loss.mean().backward()
        out = loss.detach()
    except RuntimeError as e:
        out = str(e)
    TPm._ADD_LEDGER["live"].clear()
    stats = dict(TPm.SPLIT_STATS)
    dist.destroy_process_group()
    return out, (seen[0] if seen else None), stats


def relay_graph_worker(rank, world, port, outdir):
    """One rank of the graph-captured relay test: 2 processes on cuda:0 (one TP pair), the relay's
    exchange captured in a HIP graph and replayed 20 times with fresh inputs, interleaved with
    eager exchanges: every result must equal the partner's input bit for bit (device epochs,
    csrc/kernels/xgmi_relay.hip)."""
    import os
    import pickle
    import traceback

    import torch

    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "RANK": str(rank),
                       "WORLD_SIZE": str(world)})
    res = {"ok": [], "err": None, "error_word": None, "replays": 0}
    try:
        import torch.distributed as dist
        from smdt_amd.comm import relay
        dist.init_process_group("gloo", rank=rank, world_size=world)
        torch.cuda.set_device(0)
        pg = dist.new_group(list(range(world)))
        partner = rank ^ 1
        eng = relay.XgmiRelay(pg, slot_bytes=1 << 20, sub=2, validate=True)
        n = 3 * world * (1 << 20) // 2 // 2 + 800            # bf16: 3 relay calls per exchange
        base = torch.arange(n, device="cuda", dtype=torch.float32) % 251

        def val(r, it):
            return ((base + 7.0 * r + 3.0 * it) % 509).to(torch.bfloat16)
        x = torch.empty(n, device="cuda", dtype=torch.bfloat16)
        y = torch.empty_like(x)
        for it in range(3):                                # eager: the counter advances
            x.copy_(val(rank, it))
            assert eng.exchange(x, y)
            torch.cuda.synchronize()
            res["ok"].append(bool(torch.equal(y, val(partner, it))))
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            eng.exchange(x, y)
        dist.barrier()
        for it in range(20):
            x.copy_(val(rank, 100 + it))
            g.replay()
            torch.cuda.synchronize()
            res["ok"].append(bool(torch.equal(y, val(partner, 100 + it))))
            res["replays"] += 1
            if it % 5 == 4:                                # eager calls between replays
                x.copy_(val(rank, 200 + it))
                eng.exchange(x, y)
                torch.cuda.synchronize()
                res["ok"].append(bool(torch.equal(y, val(partner, 200 + it))))
        res["error_word"] = eng.error()
        del g
        eng.close()
        dist.destroy_process_group()
    except Exception:
        res["err"] = traceback.format_exc()
    with open(os.path.join(outdir, f"r{rank}.pkl"), "wb") as f:
        pickle.dump(res, f)


def xgmi_graph_worker(rank, world, port, outdir):
    """One rank of the graph-captured xGMI-engine test: ``world`` processes on cuda:0 (real IPC
    mappings), the engine's chunked all-reduce, reduce-scatter and all-gather — the async forms
    DDP / ZeRO use, on the engine's side stream with event handles — captured ONCE in a HIP graph
    and replayed 20 times with fresh inputs, eager calls interleaved; every result exact against
    the host-computed sum (per-block device call counters, csrc/kernels/xgmi_allreduce.hip)."""
    import os
    import pickle
    import traceback

    import torch

    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "RANK": str(rank),
                       "WORLD_SIZE": str(world)})
    res = {"ok": [], "err": None, "error_word": None, "replays": 0}
    try:
        import torch.distributed as dist
        from smdt_amd.comm import xgmi
        dist.init_process_group("gloo", rank=rank, world_size=world)
        torch.cuda.set_device(0)
        eng = xgmi.XgmiAllReduce(None, region_bytes=4 << 20, blocks=16, validate=False)
        n_ar = 2 * (4 << 20) // 4 + 1024            # fp32: 3 region bands
        ns = 3 * (4 << 20) // (4 * world) + 256     # reduce-scatter / all-gather slice: 4 bands
        ar = torch.empty(n_ar, device="cuda")
        full = torch.empty(world * ns, device="cuda")
        gat = torch.empty(world * ns, device="cuda")

        def fill(it):
            ar.copy_(torch.arange(n_ar, device="cuda", dtype=torch.float32) % 89 + 7.0 * rank + it)
            full.copy_(torch.arange(world * ns, device="cuda", dtype=torch.float32) % 53 + 3.0 * rank + it)
            gat.fill_(-1.0)
            gat.view(world, ns)[rank].copy_(torch.arange(ns, device="cuda", dtype=torch.float32) + 100.0 * rank + it)

        def want(it):
            a = sum(torch.arange(n_ar, device="cuda", dtype=torch.float32) % 89 + 7.0 * r + it for r in range(world))
            f = sum(torch.arange(world * ns, device="cuda", dtype=torch.float32) % 53 + 3.0 * r + it
                    for r in range(world)).view(world, ns)[rank]
            g = torch.cat([torch.arange(ns, device="cuda", dtype=torch.float32) + 100.0 * r + it for r in range(world)])
            return a, f, g

        def step():
            h1 = eng.all_reduce_async(ar)
            h2 = eng.reduce_scatter_async(full.view(world, ns)[rank], full)
            h3 = eng.all_gather_async(gat, gat.view(world, ns)[rank])
            assert h1 is not None and h2 is not None and h3 is not None
            for h in (h1, h2, h3):
                h.wait()

        def check(it):
            torch.cuda.synchronize()
            a, f, g = want(it)
            res["ok"].append(bool(torch.equal(ar, a) and torch.equal(full.view(world, ns)[rank], f)
                                  and torch.equal(gat, g)))
        for it in range(3):                        # eager: the device call counters advance
            fill(it)
            step()
            check(it)
        fill(0)
        torch.cuda.synchronize()
        dist.barrier()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            step()
        torch.cuda.synchronize()
        dist.barrier()
        for it in range(20):
            fill(10 + it)
            g.replay()
            check(10 + it)
            res["replays"] += 1
            if it % 5 == 4:                        # eager calls between replays
                fill(100 + it)
                step()
                check(100 + it)
        res["error_word"] = eng.error()
        del g
        eng.close()
        dist.destroy_process_group()
    except Exception:
        res["err"] = traceback.format_exc()
    with open(os.path.join(outdir, f"r{rank}.pkl"), "wb") as f:
        pickle.dump(res, f)


def ddp_xgmi_graph_worker(rank, world, port, outdir, zero):
    """One rank of the DDP-level graph test: ``world`` processes on cuda:0, the framework's DDP
    over a Gloo world with an xGMI engine on real IPC mappings put in as its DP engine and
    ``xgmi_in_graph`` on: the gradient sync (``finish_grad_sync``: every bucket's all-reduce, or
    with ``zero`` its reduce-scatter) captured once and replayed with fresh gradients, the health
    check run between replays (``health_between_replays``). Every reduced value exact."""
    import os
    import pickle
    import traceback

    import torch

    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "RANK": str(rank),
                       "WORLD_SIZE": str(world)})
    res = {"ok": [], "err": None, "error_word": None, "replays": 0, "engine_calls": 0}
    try:
        import torch.distributed as dist
        from smdt_amd.comm import xgmi
        from smdt_amd.parallel import state as ps
        from smdt_amd.parallel.distributed import DistributedDataParallel as DDP
        dist.init_process_group("gloo", rank=rank, world_size=world)
        torch.cuda.set_device(0)
        ps.initialize_model_parallel(1, 1)
        torch.manual_seed(0)
        model = torch.nn.Sequential(torch.nn.Linear(256, 512), torch.nn.Linear(512, 256)).cuda()
        ddp = DDP(model, grad_dtype=torch.float32, bucket_size=40000, use_distributed_optimizer=zero)
        assert ddp.xgmi is None                        # a Gloo group: no engine of its own
        ddp.xgmi = xgmi.XgmiAllReduce(None, region_bytes=1 << 20, blocks=16, validate=False)
        ddp.xgmi_in_graph = True
        n = ddp.grad_data.numel()
        base = torch.arange(n, device="cuda", dtype=torch.float32) % 97

        def fill(it):
            ddp.grad_data.copy_(base + 4.0 * rank + it)

        def check(it):
            torch.cuda.synchronize()
            want = base + 2.0 * (world - 1) + it      # the average of the ranks' fills
            ok = True
            for b in ddp.buckets:
                s, e = ddp.shard_range(b) if zero else (b.start, b.end)
                ok = ok and torch.equal(ddp.grad_data[s:e], want[s:e])
            res["ok"].append(bool(ok))
        for it in range(2):
            fill(it)
            ddp.finish_grad_sync()
            check(it)
        calls0 = ddp.xgmi.calls
        fill(0)
        torch.cuda.synchronize()
        dist.barrier()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            ddp.finish_grad_sync()
        res["engine_calls"] = ddp.xgmi.calls - calls0   # issued into the graph
        torch.cuda.synchronize()
        dist.barrier()
        for it in range(10):
            assert ddp.health_between_replays()
            fill(10 + it)
            g.replay()
            check(10 + it)
            res["replays"] += 1
        res["error_word"] = ddp.xgmi.error()
        del g
        ddp.xgmi.close()
        dist.destroy_process_group()
    except Exception:
        res["err"] = traceback.format_exc()
    with open(os.path.join(outdir, f"r{rank}.pkl"), "wb") as f:
        pickle.dump(res, f)
