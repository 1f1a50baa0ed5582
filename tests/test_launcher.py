"""Estimator-style launcher: hyperparameter marshalling, SM_* env, metric scraping,
and BASELINE config #1 end to end — MNIST CNN DDP on CPU/gloo, world_size 2, launched through
``PyTorch(...).fit(...)`` exactly like NB1."""
import json
import os
import tarfile

import pytest
import torch

from smdt_amd.launch import hyperparameters as H
from smdt_amd.launch.metrics import MetricScraper

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_hyperparameters_sorted_and_bools_as_strings():
    cli = H.hyperparameters_to_cli({"lr": 0.1, "backend": "smddp", "bf16": False, "epochs": 2,
                                    "output_dir": "/opt/ml/model"}, remap_root="/jobs/x")
    assert cli == ["--backend", "smddp", "--bf16", "False", "--epochs", "2", "--lr", "0.1",
                   "--output_dir", "/jobs/x/model"]


def test_training_env_contract(tmp_path):
    env = H.training_env(str(tmp_path), {"epochs": 1}, {"training": str(tmp_path / "input/data/training")},
                         "train.py", num_gpus=8)
    for k in ("SM_MODEL_DIR", "SM_CHANNEL_TRAINING", "SM_HPS", "SM_NUM_GPUS", "SM_HOSTS", "SM_CURRENT_HOST",
              "SM_USER_ARGS"):
        assert k in env, k
    assert json.loads(env["SM_HPS"]) == {"epochs": 1}
    assert env["SM_NUM_GPUS"] == "8"


def test_metric_scraper_on_recipe_lines():
    sc = MetricScraper([{"Name": "train:loss", "Regex": r"Train_Loss=(.*?);"},
                        {"Name": "val:top1", "Regex": r"Val_Prec@1=(.*?):"},
                        {"Name": "nb1-broken", "Regex": r"Train Loss: (.*?),"}])
    for line in ("Epoch: [1][10/20]\tTrain_Time=0.123: avg-0.130, Train_Speed=1234: avg-1200, "
                 "Train_Loss=0.5678: avg-0.6, Train_Prec@1=80.0: avg-79.0", "Val_Prec@1=91.000: top5",
                 "Train Epoch: 1 [0/6000 (0%)]\tLoss: 2.300000"):
        sc.feed(line)
    assert sc.last("val:top1") == 91.0
    assert sc.series["nb1-broken"] == []        # the reference regex never matches (kept visible)


@pytest.mark.slow
def test_mnist_ddp_gloo_world2_through_estimator(tmp_path):
    """BASELINE config #1: the NB1 call sequence (PyTorch estimator, mpi distribution, 2 processes)."""
    from smdt_amd.data.mnist import write_synthetic_mnist
    from smdt_amd.launch import LocalSession, PyTorch
    data = tmp_path / "mnist"
    write_synthetic_mnist(str(data), n_train=512, n_test=128)
    sess = LocalSession(root=str(tmp_path / "jobs"))
    est = PyTorch(entry_point="pytorch_mnist_ddp.py",
                  source_dir=os.path.join(REPO, "recipes", "1_training_mnist_ddp"),
                  role="arn:aws:iam::000000000000:role/local", framework_version="2.0.0", py_version="py310",
                  instance_count=1, instance_type="local", sagemaker_session=sess,
                  distribution={"mpi": {"enabled": True, "processes_per_host": 2}},
                  hyperparameters={"epochs": 1, "backend": "gloo", "batch-size": 64, "lr": 1.0,
                                   "test-batch-size": 128, "log-interval": 2},
                  metric_definitions=[{"Name": "test:accuracy", "Regex": r"Accuracy: \d+/\d+ \((\d+)%\)"}],
                  disable_profiler=True, debugger_hook_config=False, max_run=600)
    est.fit({"training": f"file://{data}"}, job_name="mnist-gloo-ws2")
    job = sess.job_dir("mnist-gloo-ws2")
    log = open(os.path.join(job, "logs", "job.log")).read()
    assert "Test set: Average loss" in log and "over 2 rank(s)" in log
    assert os.path.exists(est.model_data)
    with tarfile.open(est.model_data) as t:
        names = t.getnames()
    assert any(n.endswith("mnist_cnn.pt") for n in names)
    metrics = json.load(open(os.path.join(job, "metrics.json")))
    assert metrics["test:accuracy"], metrics
    with tarfile.open(est.model_data) as t:
        t.extractall(tmp_path / "model")
    sd = torch.load(next((tmp_path / "model").rglob("mnist_cnn.pt")), weights_only=True)
    assert "module.conv1.weight" in sd


@pytest.mark.parametrize("reqs,ok", [("albumentations\nnumpy>=1.20  # comment\n", True),
                                     ("numpy\ndefinitely-not-a-module-xyz==1.0\n", False)])
def test_source_dir_requirements_txt(tmp_path, reqs, ok):
    """E6: a source_dir with requirements.txt logs the toolkit's "Installing dependencies from
    requirements.txt" line; offline, each requirement must be importable or provided in-tree
    (albumentations -> the GPU augmentation), else the job fails before the entry point runs,
    naming the missing module (reference 2_training_oxford-pet_ddp/requirements.txt:1)."""
    from smdt_amd.launch import LocalSession, PyTorch
    src = tmp_path / "src"
    src.mkdir()
    (src / "requirements.txt").write_text(reqs)
    (src / "train.py").write_text("print('ENTRY POINT RAN')\n")
    sess = LocalSession(root=str(tmp_path / "jobs"))
    est = PyTorch(entry_point="train.py", source_dir=str(src), role="r", framework_version="2.0.0",
                  py_version="py310", instance_count=1, instance_type="local", sagemaker_session=sess)
    try:
        est.fit(job_name="reqs")
    except Exception as e:          # a failed job may raise from fit(); the log is what counts
        assert not ok, e
    log = open(os.path.join(sess.job_dir("reqs"), "logs", "job.log")).read()
    assert "Installing dependencies from requirements.txt" in log
    if ok:
        assert "albumentations: provided in-tree" in log and "ENTRY POINT RAN" in log
    else:
        assert "definitely_not_a_module_xyz" in log and "ENTRY POINT RAN" not in log
        status = json.load(open(os.path.join(sess.job_dir("reqs"), "status.json")))
        assert status["state"] == "Failed"
