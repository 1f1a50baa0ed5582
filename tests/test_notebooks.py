"""The notebooks' call sequences through the Estimator.

Each test builds the estimator with the notebook's own hyperparameter dict — only sizes are
shrunk so the job runs on two CPU processes over gloo — its ``distribution``, its channel names,
``.fit(inputs=..., job_name=...)``, and then checks what the notebook reads afterwards: the
artefacts inside ``model.tar.gz`` and the metric regexes against the job's stdout.

* NB2 (/root/reference/2_training_oxford-pet_ddp.ipynb cells 20-27): ``smdistributed``
  dataparallel, channel ``training``, ``model_history.p`` + ``checkpoint.pth`` in the model dir,
  the notebook's eight ``Train_*`` / ``Test_*`` metric regexes.
* NB3 (3_training_megatron-lm.ipynb cells 11-20): ``mpi``, ``/opt/ml/...`` data / vocab / save
  paths, channels ``dataset`` and ``model_weight``; Megatron checkpoint layout
  ``iter_XXXXXXX/mp_rank_*/model_optim_rng.pt`` + ``latest_checkpointed_iteration.txt``.
* NB4 (4_training_alpaca_deepspeed.ipynb cells 14-23): ``mpi``, channels ``training`` and
  ``cache_dir``, the DeepSpeed JSON under ``/opt/ml/code/configs``; ZeRO layout
  ``global_stepN/...`` + ``latest`` and the HF trainer state.
"""
import json
import os
import tarfile

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

NB2_HPS = {'model_name': 'swin_b', 'num-classes': 37, 'height': 128, 'width': 128, 'num-epochs': 15,
           'batch-size': 80, 'test-batch-size': 200, 'lr': 0.0001, 'backend': 'smddp'}
NB2_METRICS = [
    {'Name': 'train:Time', 'Regex': 'Train_Time=(.*?):'},
    {'Name': 'train:Loss', 'Regex': 'Train_Loss=(.*?):'},
    {'Name': 'train:Prec@1', 'Regex': 'Train_Prec@1=(.*?):'},
    {'Name': 'train:Prec@5', 'Regex': 'Train_Prec@5=(.*?):'},
    {'Name': 'test:Time', 'Regex': 'Test_Time=(.*?):'},
    {'Name': 'test:Loss', 'Regex': 'Test_Loss=(.*?):'},
    {'Name': 'test:Prec@1', 'Regex': 'Test_Prec@1=(.*?):'},
    {'Name': 'test:Prec@5', 'Regex': 'Test_Prec@5=(.*?):'},
]
NB3_HPS = {
    'num-layers': 12, 'hidden-size': 768, 'num-attention-heads': 12, 'seq-length': 1024,
    'max-position-embeddings': 1024, 'micro-batch-size': 12, 'global-batch-size': 192, 'lr': 0.0005,
    'train-iters': 4000, 'lr-decay-iters': 150000, 'lr-decay-style': 'cosine', 'lr-warmup-iters': 2000,
    'weight-decay': .1, 'adam-beta2': .999, 'fp16': 'true', 'log-interval': 10, 'save-interval': 2000,
    'eval-interval': 200, 'eval-iters': 10,
    'data-path': '/opt/ml/input/data/dataset/codeparrot_content_document',
    'vocab-file': '/opt/ml/input/data/dataset/gpt2-vocab.json',
    'merge-file': '/opt/ml/input/data/dataset/gpt2-merges.txt',
    'save': '/opt/ml/model/', 'tensor-model-parallel-size': 4, 'pipeline-model-parallel-size': 1}
NB4_HPS = {
    'model_name_or_path': 'facebook/opt-125m', 'data_path': '/opt/ml/input/data/training/alpaca_data.json',
    'bf16': False, 'output_dir': '/opt/ml/model', 'num_train_epochs': 1, 'per_device_train_batch_size': 4,
    'per_device_eval_batch_size': 4, 'gradient_accumulation_steps': 8, 'evaluation_strategy': 'no',
    'save_strategy': 'steps', 'save_steps': 2000, 'save_total_limit': 1, 'learning_rate': 2e-5,
    'weight_decay': 0., 'warmup_ratio': 0.03, 'deepspeed': "/opt/ml/code/configs/default_offload_opt_param.json",
    'tf32': False, 'cache_dir': '/opt/ml/input/data/cache_dir', 'report_to': 'none'}


def _estimator(tmp_path, entry, source, hps, distribution, metrics=None):
    from smdt_amd.launch import LocalSession, PyTorch
    sess = LocalSession(root=str(tmp_path / "jobs"))
    sess.config = {'local': {'local_code': True}}
    est = PyTorch(entry_point=entry, source_dir=os.path.join(REPO, "recipes", source),
                  role="arn:aws:iam::000000000000:role/local", framework_version='1.13.1', py_version='py39',
                  instance_count=2, instance_type='local', distribution=distribution,
                  metric_definitions=metrics, disable_profiler=True, debugger_hook_config=False,
                  max_run=3600, hyperparameters=hps, sagemaker_session=sess,
                  processes_per_host=2, environment={"OMP_NUM_THREADS": "2", "CUDA_VISIBLE_DEVICES": ""})
    return sess, est


def _tar_names(path):
    with tarfile.open(path) as t:
        return t.getnames()


@pytest.mark.slow
def test_nb2_oxford_smddp_through_estimator(tmp_path):
    from smdt_amd.data.image_folder import write_synthetic_image_folder
    data = tmp_path / "oxford"
    write_synthetic_image_folder(str(data / "train"), num_classes=4, per_class=6, size=64, seed=0)
    write_synthetic_image_folder(str(data / "val"), num_classes=4, per_class=2, size=64, seed=1)
    hps = {**NB2_HPS, 'height': 64, 'width': 64, 'num-epochs': 1, 'batch-size': 4, 'test-batch-size': 4,
           'max-steps': 2, 'num-workers': 0, 'log-interval': 1, 'pretrained': False}
    distribution = {}
    if hps['backend'] == 'nccl':
        distribution["mpi"] = {"enabled": True}
    elif hps['backend'] == 'smddp':
        distribution["smdistributed"] = {"dataparallel": {"enabled": True}}
    sess, est = _estimator(tmp_path, 'pytorch_oxford_ddp.py', '2_training_oxford-pet_ddp', hps, distribution,
                           NB2_METRICS)
    est.fit(inputs={'training': f"file://{data}"}, job_name='oxford-local-0101-00000000000000')
    job = sess.job_dir('oxford-local-0101-00000000000000')
    log = open(os.path.join(job, "logs", "job.log")).read()
    assert "2 process(es)" in log
    names = _tar_names(est.model_data)
    assert any(n.endswith("model_history.p") for n in names) and any(n.endswith("checkpoint.pth") for n in names)
    with tarfile.open(est.model_data) as t:
        t.extractall(tmp_path / "model")
    hist = json.load(open(next((tmp_path / "model").rglob("model_history.p"))))   # the notebook's json.load
    for k in ('epoch', 'losses', 'top1', 'top5', 'val_avg_epoch', 'val_avg_losses', 'val_avg_top1', 'val_avg_top5'):
        assert k in hist, k
    metrics = json.load(open(os.path.join(job, "metrics.json")))
    for m in NB2_METRICS:
        assert metrics[m['Name']], (m, log[-3000:])


def _megatron_dataset(root):
    from smdt_amd.data.indexed_dataset import write_synthetic_corpus
    os.makedirs(root, exist_ok=True)
    vocab = {chr(c): c - 33 for c in range(33, 127)}           # a tiny byte-level BPE vocabulary
    vocab["<|endoftext|>"] = len(vocab)
    with open(os.path.join(root, "gpt2-vocab.json"), "w") as f:
        json.dump(vocab, f)
    with open(os.path.join(root, "gpt2-merges.txt"), "w") as f:
        f.write("#version: 0.2\n")
    write_synthetic_corpus(os.path.join(root, "codeparrot_content_document"), num_docs=64, vocab_size=len(vocab),
                           mean_len=80)


@pytest.mark.slow
def test_nb3_megatron_mpi_through_estimator(tmp_path):
    _megatron_dataset(str(tmp_path / "dataset"))
    weights = tmp_path / "model_weight"
    weights.mkdir()
    hps = {**NB3_HPS, 'num-layers': 2, 'hidden-size': 64, 'num-attention-heads': 4, 'seq-length': 64,
           'max-position-embeddings': 64, 'micro-batch-size': 2, 'global-batch-size': 4, 'train-iters': 4,
           'lr-warmup-iters': 1, 'log-interval': 1, 'save-interval': 2, 'eval-interval': 2, 'eval-iters': 1,
           'tensor-model-parallel-size': 2}
    distribution = {"mpi": {"enabled": True}}
    sess, est = _estimator(tmp_path, 'pretrain_gpt.py', '3_training_megatron-lm', hps, distribution,
                           [{'Name': 'train:lm-loss', 'Regex': r'lm loss: ([0-9.E+-]+)'}])
    est.fit(inputs={'dataset': f"file://{tmp_path / 'dataset'}", 'model_weight': f"file://{weights}"},
            job_name='megatron-lm-local-0101-00000000000000')
    names = _tar_names(est.model_data)
    assert any(n.endswith("latest_checkpointed_iteration.txt") for n in names), names
    for it in ("iter_0000002", "iter_0000004"):
        for tp in ("mp_rank_00", "mp_rank_01"):
            assert any(n.endswith(f"{it}/{tp}/model_optim_rng.pt") for n in names), (it, tp, names)
    job = sess.job_dir('megatron-lm-local-0101-00000000000000')
    log = open(os.path.join(job, "logs", "job.log")).read()
    assert "world size 2" in log.lower() or "tensor-model-parallel size: 2" in log.lower() or "tp 2" in log.lower()
    metrics = json.load(open(os.path.join(job, "metrics.json")))
    assert len(metrics['train:lm-loss']) >= 4


@pytest.mark.slow
def test_nb4_alpaca_deepspeed_through_estimator(tmp_path):
    from smdt_amd.data import sft
    data = tmp_path / "training"
    data.mkdir()
    sft.write_synthetic_alpaca(str(data / "alpaca_data.json"), 48)
    cache = tmp_path / "cache_dir"
    (cache / "facebook" / "opt-125m").mkdir(parents=True)
    tiny = {"model_type": "opt", "hidden_size": 64, "num_hidden_layers": 2, "num_attention_heads": 4,
            "ffn_dim": 128, "max_position_embeddings": 512, "vocab_size": 50272, "word_embed_proj_dim": 64,
            "do_layer_norm_before": True, "activation_function": "relu", "pad_token_id": 1, "bos_token_id": 2,
            "eos_token_id": 2, "enable_bias": True, "layer_norm_elementwise_affine": True}
    json.dump(tiny, open(cache / "facebook" / "opt-125m" / "config.json", "w"))
    hps = {**NB4_HPS, 'per_device_train_batch_size': 2, 'gradient_accumulation_steps': 2, 'save_steps': 4,
           'model_max_length': 64}
    distribution = {"mpi": {"enabled": True}}
    sess, est = _estimator(tmp_path, 'train.py', '4_training_alpaca_deepspeed', hps, distribution,
                           [{'Name': 'train:loss', 'Regex': r"'train_loss': ([0-9.]+)"}])
    est.fit(inputs={'training': f"file://{data}", 'cache_dir': f"file://{cache}"},
            job_name='alpaca-local-0101-00000000000000')
    names = _tar_names(est.model_data)
    assert any(n.endswith("/latest") or n == "latest" for n in names), names
    assert any("global_step" in n for n in names), names
    assert any(n.endswith("trainer_state.json") for n in names), names
    job = sess.job_dir('alpaca-local-0101-00000000000000')
    metrics = json.load(open(os.path.join(job, "metrics.json")))
    log = open(os.path.join(job, "logs", "job.log")).read()
    assert metrics['train:loss'], log[-3000:]
    assert "[zero.Init]" in log, log[-3000:]       # stage 3 config: partitioned construction
