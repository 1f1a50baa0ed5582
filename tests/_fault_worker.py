"""Tiny multi-rank job used by the fail-fast / fault-injection tests (run under the supervisor)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from smdt_amd.utils.debug import StepWatchdog, maybe_inject_fault  # noqa: E402


def main():
    mode = sys.argv[1] if len(sys.argv) > 1 else "steps"
    if mode == "watchdog":
        with StepWatchdog(1.0, abort=True):
            time.sleep(30)
        return
    dist.init_process_group("gloo", timeout=__import__("datetime").timedelta(seconds=120))
    t = torch.ones(4)
    for step in range(1, 6):
        maybe_inject_fault(step)
        dist.all_reduce(t)
    dist.destroy_process_group()
    print(f"rank {os.environ['RANK']} done", flush=True)


if __name__ == "__main__":
    main()
