"""MIOpen's user find / perf databases for the Oxford-Pet vision recipe, seeded from the repo.

A fresh process on a fresh MI355X spends its first ResNet-50 steps in MIOpen's Find (benchmarking
every applicable solver per convolution config) and compiling the winners: 84 s of start-up
before the first timed step at 224 x 224 x 64 bf16 NHWC, against 22 s when MIOpen finds its user
database already filled and only compiles (the steady-state rate is the same, ~4,750 img/s:
profiles/r5_miopen/README.md). ``utils/miopen_db/`` holds those two TEXT databases as MIOpen wrote
them on gfx950 (256 CUs) for the recipe's ResNet-50 and swin_b shapes (the solver picked per
config and its measured time; no code). ``seed_user_db()`` puts them where MIOpen looks before
the process's first convolution, without overwriting anything MIOpen already wrote there; MIOpen
ignores files of another architecture or version by name.
"""
from __future__ import annotations

import os
import shutil

_SHIPPED = os.path.join(os.path.dirname(os.path.abspath(__file__)), "miopen_db")


def shipped_files():
    return sorted(f for f in os.listdir(_SHIPPED) if f.endswith(".txt")) if os.path.isdir(_SHIPPED) else []


def seed_user_db(target: str = None) -> str:
    """Copy the shipped databases into MIOpen's user database directory (``MIOPEN_USER_DB_PATH``
    if set, else ``~/.cache/smdt_amd/miopen``, which then becomes ``MIOPEN_USER_DB_PATH`` for this
    process and its children); files already there are kept. Call before the first convolution.
    Returns the directory, or "" when it cannot be written (MIOpen then works as without it)."""
    d = target or os.environ.get("MIOPEN_USER_DB_PATH") or os.path.join(
        os.path.expanduser("~"), ".cache", "smdt_amd", "miopen")
    try:
        os.makedirs(d, exist_ok=True)
        for f in shipped_files():
            dst = os.path.join(d, f)
            if not os.path.exists(dst):
                shutil.copyfile(os.path.join(_SHIPPED, f), dst)
    except OSError:
        return ""
    os.environ["MIOPEN_USER_DB_PATH"] = d
    return d
