"""Job environment contract: hyperparameter serialisation, SM_* / OMPI_* variables, /opt/ml paths.

Reproduces what the SageMaker training toolkit hands to a training script (log
evidence NB1:679 `SM_USER_ARGS`, NB1:686 mpirun env, NB4:877):
  * hyperparameters dict -> ``--key value`` CLI **sorted by key**; booleans become the strings
    ``True`` / ``False``; every hyperparameter is also exported as ``SM_HP_<KEY>`` and the whole
    dict as JSON in ``SM_HPS``;
  * channels -> ``/opt/ml/input/data/<channel>`` exported as ``SM_CHANNEL_<CHANNEL>``;
  * ``SM_MODEL_DIR``, ``SM_OUTPUT_DATA_DIR``, ``SM_HOSTS``, ``SM_CURRENT_HOST``, ``SM_NUM_GPUS``,
    ``SM_TRAINING_ENV`` ...;
  * per rank: ``OMPI_COMM_WORLD_{RANK,SIZE,LOCAL_RANK,LOCAL_SIZE}`` (+ torchrun's
    RANK/LOCAL_RANK/WORLD_SIZE/MASTER_ADDR/MASTER_PORT).

The job root replaces ``/opt/ml``: absolute ``/opt/ml/...`` strings in hyperparameters (the
reference recipes hard-code e.g. ``'save': '/opt/ml/model/'``, NB3:399-428) are remapped into it.
"""
from __future__ import annotations

import json
import os
from typing import Dict, List, Mapping, Optional

OPT_ML = "/opt/ml"


def _fmt(v) -> str:
    if isinstance(v, bool):
        return "True" if v else "False"
    if isinstance(v, (dict, list)):
        return json.dumps(v)
    return str(v)


def hyperparameters_to_cli(hps: Mapping, remap_root: Optional[str] = None) -> List[str]:
    """{'b': 1, 'a': True} -> ['--a', 'True', '--b', '1'] (sorted by key, like the toolkit)."""
    out: List[str] = []
    for k in sorted(hps):
        v = _fmt(hps[k])
        if remap_root:
            v = remap_opt_ml(v, remap_root)
        out += [f"--{k}", v]
    return out


def remap_opt_ml(value: str, root: str) -> str:
    if isinstance(value, str) and (value == OPT_ML or value.startswith(OPT_ML + "/")):
        return os.path.join(root, value[len(OPT_ML) + 1:]) if value != OPT_ML else root
    return value


def job_paths(root: str) -> Dict[str, str]:
    return {
        "root": root,
        "code": os.path.join(root, "code"),
        "model": os.path.join(root, "model"),
        "input": os.path.join(root, "input"),
        "input_data": os.path.join(root, "input", "data"),
        "input_config": os.path.join(root, "input", "config"),
        "output": os.path.join(root, "output"),
        "output_data": os.path.join(root, "output", "data"),
        "checkpoints": os.path.join(root, "checkpoints"),
    }


def training_env(root: str, hps: Mapping, channels: Mapping[str, str], entry_point: str, num_gpus: int,
                 hosts=("algo-1",), current_host="algo-1", job_name="job", module_dir: Optional[str] = None,
                 network_interface="lo") -> Dict[str, str]:
    """The SM_* environment for one job (identical on every rank)."""
    p = job_paths(root)
    user_args = hyperparameters_to_cli(hps, remap_root=root)
    env = {
        "SM_MODEL_DIR": p["model"],
        "SM_OUTPUT_DIR": p["output"],
        "SM_OUTPUT_DATA_DIR": p["output_data"],
        "SM_OUTPUT_INTERMEDIATE_DIR": os.path.join(p["output"], "intermediate"),
        "SM_INPUT_DIR": p["input"],
        "SM_INPUT_CONFIG_DIR": p["input_config"],
        "SM_CHANNELS": json.dumps(sorted(channels)),
        "SM_HOSTS": json.dumps(list(hosts)),
        "SM_CURRENT_HOST": current_host,
        "SM_NUM_GPUS": str(num_gpus),
        "SM_NUM_CPUS": str(os.cpu_count() or 1),
        "SM_NETWORK_INTERFACE_NAME": network_interface,
        "SM_LOG_LEVEL": "20",
        "SM_USER_ENTRY_POINT": entry_point,
        "SM_MODULE_DIR": module_dir or p["code"],
        "SM_MODULE_NAME": os.path.splitext(os.path.basename(entry_point))[0],
        "SM_HPS": json.dumps({k: hps[k] for k in sorted(hps)}),
        "SM_USER_ARGS": json.dumps(user_args),
        "SM_FRAMEWORK_PARAMS": "{}",
        "SM_CHECKPOINT_DIR": p["checkpoints"],
        "SM_JOB_NAME": job_name,
    }
    for ch, path in channels.items():
        env[f"SM_CHANNEL_{ch.upper()}"] = path
    for k, v in hps.items():
        env[f"SM_HP_{k.upper().replace('-', '_')}"] = remap_opt_ml(_fmt(v), root)
    te = {
        "channel_input_dirs": dict(channels), "current_host": current_host, "hosts": list(hosts),
        "hyperparameters": dict(hps), "job_name": job_name, "model_dir": p["model"], "num_gpus": num_gpus,
        "output_data_dir": p["output_data"], "user_entry_point": entry_point, "module_dir": env["SM_MODULE_DIR"],
    }
    env["SM_TRAINING_ENV"] = json.dumps(te, default=str)
    return env


def rank_env(rank: int, local_rank: int, world: int, local_world: int, master_addr="127.0.0.1",
             master_port=29500, node_rank=0) -> Dict[str, str]:
    """mpirun-style (OMPI_COMM_WORLD_*) plus torchrun-style rank variables."""
    return {
        "OMPI_COMM_WORLD_RANK": str(rank), "OMPI_COMM_WORLD_SIZE": str(world),
        "OMPI_COMM_WORLD_LOCAL_RANK": str(local_rank), "OMPI_COMM_WORLD_LOCAL_SIZE": str(local_world),
        "OMPI_COMM_WORLD_NODE_RANK": str(node_rank),
        "RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(local_rank),
        "LOCAL_WORLD_SIZE": str(local_world), "NODE_RANK": str(node_rank),
        "MASTER_ADDR": master_addr, "MASTER_PORT": str(master_port),
    }
