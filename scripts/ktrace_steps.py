"""Per-kernel breakdown of the LAST training step in a rocprofv3 kernel trace.

Steps are delimited by the optimizer's adam kernels (a cluster of consecutive adam launches ends
each step). Usage: python scripts/ktrace_steps.py <kernel_trace.csv> [top_n] [--step -1]
"""
import csv
import re
import sys
from collections import defaultdict


def short(name):
    n = re.sub(r"\(.*", "", name)
    n = re.sub(r"^void ", "", n)
    return n[:110]


def main():
    path = sys.argv[1]
    top = int(sys.argv[2]) if len(sys.argv) > 2 and sys.argv[2].isdigit() else 40
    which = -1
    if "--step" in sys.argv:
        which = int(sys.argv[sys.argv.index("--step") + 1])
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    adam = [i for i, r in enumerate(rows) if "adam_kernel" in r[2] or "adam_batch_kernel" in r[2]]
    ends = []
    for j, i in enumerate(adam):
        if j + 1 == len(adam) or adam[j + 1] - i > 50:
            ends.append(i)
    if len(ends) < 2:
        sys.exit("need at least two optimizer steps in the trace")
    e = ends[which]
    s = ends[which - 1] + 1
    step = rows[s:e + 1]
    wall = (step[-1][1] - step[0][0]) / 1e6
    agg = defaultdict(lambda: [0, 0.0])
    for a, b, n in step:
        k = short(n)
        agg[k][0] += 1
        agg[k][1] += (b - a) / 1e6
    busy = sum(v[1] for v in agg.values())
    print(f"step {which}: {len(step)} kernels, wall {wall:.2f} ms, kernel-busy {busy:.2f} ms "
          f"(gaps {wall - busy:.2f} ms)")
    for k, (c, t) in sorted(agg.items(), key=lambda x: -x[1][1])[:top]:
        print(f"{t:8.3f} ms {100 * t / busy:5.1f}%  n={c:4d}  {k}")


if __name__ == "__main__":
    main()
