"""stanford_alpaca ``utils`` helpers used by the recipe (``jload``/``jdump``)."""
import os
import sys

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")))

from smdt_amd.data.sft import jdump, jload  # noqa: E402,F401
