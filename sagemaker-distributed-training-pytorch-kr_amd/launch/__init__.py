"""Estimator-compatible launch API (``sagemaker``-style) for one MI355X node.

    from smdt_amd.launch import Session, LocalSession, PyTorch, FileSystemInput, get_execution_role
"""
from .estimator import Estimator, FileSystemInput, LocalSession, PyTorch, Session, get_execution_role  # noqa: F401
from .hyperparameters import hyperparameters_to_cli, rank_env, training_env  # noqa: F401
from .metrics import MetricScraper  # noqa: F401
