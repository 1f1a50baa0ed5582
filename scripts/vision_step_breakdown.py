"""Per-category kernel time of the LAST training step of a bench_vision.py rocprofv3 kernel trace.

Steps end with torch's fused Adam launches (a cluster of ``FusedAdam`` / ``multi_tensor_apply``
kernels); the categories are conv (MIOpen / CK / igemm / naive convolution kernels), batch-norm,
GEMM (hipBLASLt / rocBLAS), optimizer, augmentation-and-elementwise (at::native kernels), other.
Also prints the step's wall time between the two Adam clusters and the device idle time in it.

usage: python scripts/vision_step_breakdown.py <kernel_trace.csv>
"""
import csv
import re
import sys
from collections import defaultdict


def category(name: str) -> str:
    n = name.lower()
    if "adam" in n or "multi_tensor" in n:
        return "optimizer"
    if "batchnorm" in n or "bnfwd" in n or "bnbwd" in n:
        return "batch-norm"
    if any(k in n for k in ("conv", "igemm", "miopensp3", "grouped_conv", "batched_gemm_xdl")):
        return "convolution"
    if "cijk" in n or "gemm" in n:
        return "gemm"
    if "at::native" in n or "elementwise" in n or "reduce_kernel" in n:
        return "elementwise / augmentation (at::native)"
    return "other"


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    adam = [i for i, r in enumerate(rows) if "adam" in r["Kernel_Name"].lower()]
    clusters = []
    for i in adam:
        if clusters and i - clusters[-1][-1] <= 5:
            clusters[-1].append(i)
        else:
            clusters.append([i])
    if len(clusters) < 2:
        raise SystemExit("need two optimizer steps in the trace")
    s, e = clusters[-2][-1] + 1, clusters[-1][-1]
    t0, t1 = int(rows[s]["Start_Timestamp"]), int(rows[e]["End_Timestamp"])
    per, cnt, busy = defaultdict(float), defaultdict(int), 0.0
    top = defaultdict(float)
    for r in rows[s:e + 1]:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        c = category(r["Kernel_Name"])
        per[c] += d
        cnt[c] += 1
        busy += d
        top[re.sub(r"\(.*", "", r["Kernel_Name"])[:90]] += d
    wall = (t1 - t0) / 1e6
    print(f"last step: {e - s + 1} kernels, wall {wall:.2f} ms (first kernel .. last Adam kernel), "
          f"kernel-busy {busy:.2f} ms, device idle {wall - busy:.2f} ms")
    for c, v in sorted(per.items(), key=lambda kv: -kv[1]):
        print(f"  {v:8.3f} ms  {100 * v / busy:5.1f}%  n={cnt[c]:5d}  {c}")
    print("top kernels:")
    for k, v in sorted(top.items(), key=lambda kv: -kv[1])[:12]:
        print(f"  {v:8.3f} ms  {k}")


if __name__ == "__main__":
    main()
