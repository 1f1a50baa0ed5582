"""Estimator-compatible job API that runs training jobs on the local MI355X node.

Keeps the notebooks' call sequence::

    sess = Session(); bucket = sess.default_bucket()
    uri = sess.upload_data(path=local_dir, bucket=bucket, key_prefix="mnist")
    est = PyTorch(entry_point="pytorch_mnist_ddp.py", source_dir="1_training_mnist_ddp",
                  role=get_execution_role(), framework_version="2.0.0", py_version="py310",
                  instance_count=1, instance_type="local_gpu",
                  distribution={"mpi": {"enabled": True}}, hyperparameters={...},
                  metric_definitions=[...], max_run=3600, sagemaker_session=sess)
    est.fit(inputs={"training": uri}, job_name="mnist-ddp", wait=True)
    est.model_data          # -> <job>/output/model.tar.gz

There is no AWS: ``s3://bucket/prefix`` URIs resolve into the session's local object store,
``file://`` URIs and ``FileSystemInput`` directories are used in place, and every rank runs on
this node under the native supervisor (one process per GPU, ``OMPI_COMM_WORLD_*`` contract,
fail-fast + process-group cleanup, ``max_run`` wall clock). Cloud-only kwargs (role, subnets,
image_uri, debugger/profiler switches, ...) are accepted and recorded.
"""
from __future__ import annotations

import datetime
import json
import os
import shutil
import socket
import subprocess
import sys
import tarfile
import threading
import time
from typing import Dict, List, Optional, Union

from .hyperparameters import hyperparameters_to_cli, job_paths, rank_env, remap_opt_ml, training_env
from .metrics import MetricScraper

_REPO_ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def get_execution_role(*_a, **_k) -> str:
    return "arn:local:iam::000000000000:role/smdt-local"


def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _gpu_count() -> int:
    try:
        import torch
        return torch.cuda.device_count()  # does not initialise the GPU on this image
    except Exception:
        return 0


class FileSystemInput:
    """EFS / FSx channel (NB3:366-378): a directory already visible on the node."""

    def __init__(self, file_system_id=None, file_system_type="FSxLustre", directory_path="/",
                 file_system_access_mode="ro", content_type=None):
        self.file_system_id = file_system_id
        self.file_system_type = file_system_type
        self.directory_path = directory_path
        self.file_system_access_mode = file_system_access_mode

    def local_path(self):
        return self.directory_path


class Session:
    """Local object store + job registry (``SMDT_JOB_ROOT``, default ``~/.smdt``)."""

    def __init__(self, root: Optional[str] = None, **_kw):
        self.root = os.path.abspath(root or os.environ.get("SMDT_JOB_ROOT", os.path.expanduser("~/.smdt")))
        os.makedirs(self.root, exist_ok=True)
        self.local_mode = False

    # -- object store
    def default_bucket(self) -> str:
        return "smdt-local-bucket"

    def _obj_path(self, bucket: str, key: str = "") -> str:
        return os.path.join(self.root, "s3", bucket, key)

    def upload_data(self, path: str, bucket: Optional[str] = None, key_prefix: str = "data", **_kw) -> str:
        bucket = bucket or self.default_bucket()
        dst = self._obj_path(bucket, key_prefix)
        os.makedirs(os.path.dirname(dst.rstrip("/")), exist_ok=True)
        if os.path.isdir(path):
            if os.path.islink(dst) or os.path.isfile(dst):
                os.remove(dst)
            elif os.path.isdir(dst):
                shutil.rmtree(dst)
            # Large datasets: link instead of copying (the store is on the same node).
            os.symlink(os.path.abspath(path), dst)
            return f"s3://{bucket}/{key_prefix}"
        os.makedirs(dst, exist_ok=True)
        shutil.copy2(path, os.path.join(dst, os.path.basename(path)))
        return f"s3://{bucket}/{key_prefix}/{os.path.basename(path)}"

    def resolve(self, uri) -> str:
        if isinstance(uri, FileSystemInput):
            return uri.local_path()
        if hasattr(uri, "config") and isinstance(getattr(uri, "config"), dict):  # TrainingInput-like
            uri = uri.config.get("DataSource", {}).get("S3DataSource", {}).get("S3Uri", uri)
        if isinstance(uri, str) and uri.startswith("s3://"):
            rest = uri[5:]
            bucket, _, key = rest.partition("/")
            return self._obj_path(bucket, key)
        if isinstance(uri, str) and uri.startswith("file://"):
            return uri[7:]
        return str(uri)

    # -- jobs
    def job_dir(self, job_name: str) -> str:
        return os.path.join(self.root, "jobs", job_name)

    def logs_for_job(self, job_name: str, wait: bool = False, poll: float = 1.0):
        """Print the job log (follow it while the job runs when ``wait``)."""
        log = os.path.join(self.job_dir(job_name), "logs", "job.log")
        status = os.path.join(self.job_dir(job_name), "status.json")
        pos = 0
        while True:
            if os.path.exists(log):
                with open(log, "r", errors="replace") as f:
                    f.seek(pos)
                    chunk = f.read()
                    pos = f.tell()
                if chunk:
                    sys.stdout.write(chunk)
                    sys.stdout.flush()
            done = os.path.exists(status) and json.load(open(status)).get("state") in ("Completed", "Failed", "Stopped")
            if done or not wait:
                break
            time.sleep(poll)

    def describe_training_job(self, job_name: str) -> dict:
        p = os.path.join(self.job_dir(job_name), "status.json")
        return json.load(open(p)) if os.path.exists(p) else {"state": "Unknown"}


class LocalSession(Session):
    """``instance_type='local_gpu'`` mode (NB1:393-404). Same runner; kept for API parity."""

    def __init__(self, root=None, **kw):
        super().__init__(root, **kw)
        self.local_mode = True
        self.config = {"local": {"local_code": True}}


class Estimator:
    """Generic estimator; ``PyTorch`` below is what the notebooks use."""

    _CLOUD_ONLY = ("role", "image_uri", "subnets", "security_group_ids", "framework_version", "py_version",
                   "disable_profiler", "debugger_hook_config", "volume_size", "output_path", "checkpoint_s3_uri",
                   "use_spot_instances", "max_wait", "keep_alive_period_in_seconds", "environment_variables")

    def __init__(self, entry_point: str, source_dir: Optional[str] = None, hyperparameters: Optional[dict] = None,
                 instance_count: int = 1, instance_type: str = "local_gpu", distribution: Optional[dict] = None,
                 metric_definitions: Optional[List[dict]] = None, max_run: int = 24 * 60 * 60,
                 sagemaker_session: Optional[Session] = None, environment: Optional[dict] = None,
                 processes_per_host: Optional[int] = None, **kwargs):
        self.entry_point = entry_point
        self.source_dir = os.path.abspath(source_dir) if source_dir else None
        self.hyperparameters_ = dict(hyperparameters or {})
        self.instance_count = int(instance_count)
        self.instance_type = instance_type
        self.distribution = distribution or {}
        self.metric_definitions = metric_definitions or []
        self.max_run = max_run
        self.session = sagemaker_session or Session()
        self.environment = dict(environment or kwargs.get("environment_variables") or {})
        self.processes_per_host = processes_per_host
        self.extra = {k: v for k, v in kwargs.items()}
        self.latest_training_job = None
        self._job_name = None
        self.metrics = None
        self.status = None

    # -- public API
    def hyperparameters(self):
        return dict(self.hyperparameters_)

    def set_hyperparameters(self, **kw):
        self.hyperparameters_.update(kw)

    @property
    def model_data(self) -> Optional[str]:
        if self._job_name is None:
            return None
        return os.path.join(self.session.job_dir(self._job_name), "output", "model.tar.gz")

    def logs(self):
        if self._job_name:
            self.session.logs_for_job(self._job_name, wait=True)

    def fit(self, inputs: Optional[Union[str, Dict[str, object]]] = None, job_name: Optional[str] = None,
            wait: bool = True, logs: Union[bool, str] = True):
        if job_name is None:
            base = os.path.splitext(os.path.basename(self.entry_point))[0].replace("_", "-")
            job_name = f"{base}-{datetime.datetime.now().strftime('%Y-%m-%d-%H-%M-%S-%f')[:-3]}"
        self._job_name = job_name
        self.latest_training_job = job_name
        if isinstance(inputs, (str, FileSystemInput)):
            inputs = {"training": inputs}
        inputs = inputs or {}
        if self.instance_count != 1:
            print(f"[smdt] instance_count={self.instance_count}: this launcher drives one MI355X node; "
                  "running instance_count=1 with all local GPUs", flush=True)
        runner = _LocalJob(self, job_name, inputs)
        if wait:
            rc = runner.run(stream=bool(logs))
            if rc != 0:
                raise RuntimeError(f"training job {job_name} failed with exit status {rc}; see "
                                   f"{os.path.join(self.session.job_dir(job_name), 'logs', 'job.log')}")
        else:
            t = threading.Thread(target=runner.run, kwargs={"stream": False}, daemon=True)
            t.start()
            self._thread = t
        return self

    def wait(self):
        t = getattr(self, "_thread", None)
        if t is not None:
            t.join()


class PyTorch(Estimator):
    """``sagemaker.pytorch.PyTorch``-compatible estimator (NB1:437-455, NB3:539-560, NB4:597-616)."""


class _LocalJob:
    def __init__(self, est: Estimator, job_name: str, inputs: Dict[str, object]):
        self.est = est
        self.job_name = job_name
        self.inputs = inputs
        self.root = est.session.job_dir(job_name)

    # ------------------------------------------------------------------ setup
    def _prepare(self):
        p = job_paths(self.root)
        for k in ("code", "model", "input_data", "input_config", "output_data", "checkpoints"):
            os.makedirs(p[k], exist_ok=True)
        os.makedirs(os.path.join(self.root, "logs"), exist_ok=True)
        src = self.est.source_dir
        if src:
            dst = p["code"]
            shutil.rmtree(dst, ignore_errors=True)
            shutil.copytree(src, dst, symlinks=True, ignore=shutil.ignore_patterns("__pycache__", ".ipynb_checkpoints"))
        else:
            shutil.copy2(self.est.entry_point, p["code"])
        channels = {}
        for name, uri in self.inputs.items():
            local = self.est.session.resolve(uri)
            link = os.path.join(p["input_data"], name)
            if os.path.lexists(link):
                if os.path.islink(link) or os.path.isfile(link):
                    os.remove(link)
                else:
                    shutil.rmtree(link)
            os.symlink(os.path.abspath(local), link)
            channels[name] = link
        hps = self.est.hyperparameters_
        with open(os.path.join(p["input_config"], "hyperparameters.json"), "w") as f:
            json.dump({k: str(v) for k, v in hps.items()}, f, indent=1)
        with open(os.path.join(p["input_config"], "inputdataconfig.json"), "w") as f:
            json.dump({k: {"TrainingInputMode": "File"} for k in channels}, f, indent=1)
        return p, channels

    def _nprocs(self):
        dist = self.est.distribution or {}
        ngpu = _gpu_count()
        per_host = self.est.processes_per_host
        if per_host is None:
            per_host = (dist.get("mpi", {}) or {}).get("processes_per_host")
        enabled = any(((dist.get(k) or {}).get("enabled") for k in ("mpi", "torch_distributed", "pytorchddp")))
        sm = (dist.get("smdistributed") or {}).get("dataparallel", {}).get("enabled", False)
        if per_host is None:
            per_host = max(ngpu, 1) if (enabled or sm) else 1
        if per_host > 1 and ngpu and per_host > ngpu:
            per_host = ngpu
        return int(per_host), ngpu, sm

    def _command(self, code_dir, args):
        ep = self.est.entry_point
        if os.path.isabs(ep):
            ep = os.path.basename(ep)
        if os.path.exists(os.path.join(code_dir, "setup.py")):
            # E6: the toolkit pip-installs the source dir and runs the module; we import it in place.
            mod = os.path.splitext(ep)[0].replace("/", ".")
            return [sys.executable, "-m", mod] + args
        return [sys.executable, os.path.join(code_dir, ep)] + args

    def _write_status(self, state, **kw):
        d = {"job_name": self.job_name, "state": state, "time": time.time()}
        d.update(kw)
        with open(os.path.join(self.root, "status.json"), "w") as f:
            json.dump(d, f, indent=1)

    # ------------------------------------------------------------------ run
    def run(self, stream: bool = True) -> int:
        p, channels = self._prepare()
        nprocs, ngpu, smddp = self._nprocs()
        hps = self.est.hyperparameters_
        args = hyperparameters_to_cli(hps, remap_root=self.root)
        base_env = dict(os.environ)
        base_env.update(training_env(self.root, hps, channels, self.est.entry_point, ngpu, job_name=self.job_name))
        base_env.update({k: remap_opt_ml(str(v), self.root) for k, v in self.est.environment.items()})
        pp = [p["code"], _REPO_ROOT]
        if base_env.get("PYTHONPATH"):
            pp.append(base_env["PYTHONPATH"])
        base_env["PYTHONPATH"] = os.pathsep.join(pp)
        base_env["SMDT_ROOT"] = _REPO_ROOT
        base_env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        if smddp:
            base_env["SMDATAPARALLEL_BACKEND"] = "rccl"
        port = _free_port()
        cmd = self._command(p["code"], args)
        argvs, envs = [], []
        for r in range(nprocs):
            e = dict(base_env)
            if nprocs > 1 or (self.est.distribution or {}):
                e.update(rank_env(r, r, nprocs, nprocs, master_port=port))
            argvs.append(cmd)
            envs.append([f"{k}={v}" for k, v in e.items()])
        log_path = os.path.join(self.root, "logs", "job.log")
        req_lines, missing = check_requirements(p["code"])
        if req_lines:
            txt = "".join(f"[smdt] {ln}\n" for ln in req_lines)
            if stream:
                sys.stdout.write(txt)
        if missing:
            err = ("[smdt] ERROR: source_dir/requirements.txt names module(s) that are not importable: "
                   + ", ".join(f"{r} ({m})" for r, m in missing) + "\n")
            with open(log_path, "w") as f:
                f.write(txt + err)
            if stream:
                sys.stdout.write(err)
            self._write_status("Failed", exit_status=1, failure_reason=err.strip(), missing_requirements=missing)
            self.est.status = 1
            return 1
        scraper = MetricScraper(self.est.metric_definitions)
        self._write_status("InProgress", nprocs=nprocs, command=cmd)
        hdr = (f"[smdt] job {self.job_name}: {nprocs} process(es) on {socket.gethostname()} "
               f"(GPUs visible: {ngpu}); cmd: {' '.join(cmd)}\n")
        rfd, wfd = os.pipe()
        logf = open(log_path, "w")
        if req_lines:
            logf.write(txt)
        logf.write(hdr)
        if stream:
            sys.stdout.write(hdr)

        def pump():
            with os.fdopen(rfd, "r", errors="replace") as r:
                for line in r:
                    logf.write(line)
                    logf.flush()
                    scraper.feed(line)
                    if stream:
                        sys.stdout.write(line)
                        sys.stdout.flush()

        th = threading.Thread(target=pump, daemon=True)
        th.start()
        t0 = time.time()
        try:
            status, per_rank, first = _run_ranks(argvs, envs, grace=10.0, max_run=float(self.est.max_run or 0),
                                                 cwd=p["code"], out_fd=wfd)
        finally:
            os.close(wfd)
            th.join()
            logf.close()
        elapsed = time.time() - t0
        scraper.dump(os.path.join(self.root, "metrics.json"))
        self.est.metrics = scraper.series
        if status == 0:
            self._package_model(p)
            self._write_status("Completed", exit_status=0, billable_seconds=int(elapsed), rank_status=per_rank)
        else:
            self._write_status("Failed", exit_status=status, first_failed_rank=first, rank_status=per_rank,
                               billable_seconds=int(elapsed))
        self.est.status = status
        return status

    def _package_model(self, p):
        out = os.path.join(self.root, "output")
        os.makedirs(out, exist_ok=True)
        with tarfile.open(os.path.join(out, "model.tar.gz"), "w:gz") as tar:
            for name in sorted(os.listdir(p["model"])):
                tar.add(os.path.join(p["model"], name), arcname=name)


# Requirements the framework provides in-tree (no package index on the node): the module the
# recipe would import -> what replaces it. The Oxford recipe's albumentations pipeline runs as the
# GPU augmentation of data/augment.py (csrc/kernels/augment.hip).
PROVIDED_IN_TREE = {"albumentations": "smdt_amd.data.augment (GPU augmentation, csrc/kernels/augment.hip)"}
# distribution name -> import name where they differ
_IMPORT_NAMES = {"opencv-python": "cv2", "opencv-python-headless": "cv2", "scikit-learn": "sklearn",
                 "pillow": "PIL", "pyyaml": "yaml", "protobuf": "google.protobuf", "python-dateutil": "dateutil"}


def check_requirements(code_dir):
    """E6: the toolkit pip-installs ``source_dir/requirements.txt`` before the entry point runs
    (reference 2_training_oxford-pet_ddp/requirements.txt:1, toolkit log at
    2_training_oxford-pet_ddp.ipynb:622). Offline there is nothing to install from, so each
    requirement must already be importable or be provided in-tree (PROVIDED_IN_TREE).
    Returns (log lines, missing [(requirement, module)]); no file -> ([], [])."""
    import importlib.util
    import re
    path = os.path.join(code_dir, "requirements.txt")
    if not os.path.exists(path):
        return [], []
    lines = ["sagemaker-training-toolkit INFO     Installing dependencies from requirements.txt:",
             f"sagemaker-training-toolkit INFO     (offline: checking importability, no pip) {path}"]
    missing = []
    for raw in open(path):
        req = raw.split("#", 1)[0].strip()
        if not req or req.startswith("-"):
            continue
        name = re.split(r"[\s<>=!~;\[]", req, 1)[0].strip()
        mod = _IMPORT_NAMES.get(name.lower(), name.replace("-", "_"))
        if mod in PROVIDED_IN_TREE:
            lines.append(f"  {req}: provided in-tree by {PROVIDED_IN_TREE[mod]}")
        elif importlib.util.find_spec(mod.split(".")[0]) is not None:
            lines.append(f"  {req}: importable ({mod})")
        else:
            lines.append(f"  {req}: NOT importable (module {mod!r}) and no package index to install from")
            missing.append((req, mod))
    return lines, missing


def _run_ranks(argvs, envs, grace, max_run, cwd, out_fd):
    try:
        from .. import _runtime  # native supervisor
        return _runtime.run_ranks(argvs, envs, grace, max_run, cwd, out_fd)
    except ImportError:
        return _run_ranks_py(argvs, envs, grace, max_run, cwd, out_fd)


def _run_ranks_py(argvs, envs, grace, max_run, cwd, out_fd):
    """Pure-Python fallback with the same fail-fast semantics."""
    procs = []
    for a, e in zip(argvs, envs):
        env = dict(kv.split("=", 1) for kv in e)
        procs.append(subprocess.Popen(a, env=env, cwd=cwd, stdout=out_fd, stderr=out_fd, start_new_session=True))
    t0 = time.time()
    status, first = 0, -1
    codes = [None] * len(procs)
    killing = False
    while any(c is None for c in codes):
        for i, pr in enumerate(procs):
            if codes[i] is None and pr.poll() is not None:
                rc = pr.returncode
                codes[i] = rc if rc >= 0 else 128 - rc
                if codes[i] != 0 and first < 0 and not killing:
                    first, status = i, codes[i]
        if not killing and (first >= 0 or (max_run and time.time() - t0 > max_run)):
            if status == 0:
                status = 124
            for pr in procs:
                if pr.poll() is None:
                    pr.terminate()
            killing = True
            deadline = time.time() + grace
        if killing and time.time() > deadline:
            for pr in procs:
                if pr.poll() is None:
                    pr.kill()
        time.sleep(0.05)
    return status, codes, first
