"""Recipe-local model module (the reference's training script does `from model_def import Net`,
/root/reference/1_training_mnist_ddp/pytorch_mnist_ddp.py:31). Re-exports the framework model."""
import os
import sys

_HERE = os.path.dirname(os.path.abspath(__file__))
for _cand in (os.path.join(_HERE, "..", ".."), os.environ.get("SMDT_ROOT", "")):
    if _cand and os.path.isdir(os.path.join(_cand, "smdt_amd")) and _cand not in sys.path:
        sys.path.insert(0, os.path.abspath(_cand))

from smdt_amd.models.mnist import Net  # noqa: E402,F401
