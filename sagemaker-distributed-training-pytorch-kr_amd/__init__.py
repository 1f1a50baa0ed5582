"""smdt_amd: an MI355X-native (gfx950 / CDNA4) distributed-training framework with the
capabilities of aws-samples/sagemaker-distributed-training-pytorch-kr.

Layers: ``launch`` (Estimator-compatible job API), ``comm`` (process
bootstrap, RCCL/xGMI), ``parallel`` (DDP / TP / SP / PP / ZeRO), ``ops`` (HIP kernel library),
``models`` (MNIST CNN, ResNet, GPT, LLaMA/OPT), ``optim``, ``data``, ``train`` (Megatron-style
pretrain loop, HF-style SFT trainer), ``utils``.
"""
import torch  # noqa: F401  (loads the HIP runtime before any smdt_amd extension)

__version__ = "0.1.0"
