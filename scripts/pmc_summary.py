"""Summarise rocprofv3 --pmc counter_collection.csv files: per kernel (short name), the mean of
each counter over dispatches, plus derived ratios (MFMA busy %, VALU/MFMA instruction ratio,
wait fractions). usage: python scripts/pmc_summary.py gpurun_out/pmc/p1 gpurun_out/pmc/p2"""
import csv
import glob
import os
import re
import sys
from collections import defaultdict


def short(n):
    n = re.sub(r"\(.*", "", n)
    m = re.search(r"(fwd_kernel|bwd_dkdv_kernel|bwd_dq_kernel|delta_kernel|wgrad_kernel)[^,]*", n)
    if m:
        d = re.search(r"ILi(\d+)ELb(\d)ELb(\d)", n)
        return m.group(1) + (f"<D{d.group(1)},causal{d.group(2)},drop{d.group(3)}>" if d else "")
    return n[:60]


def main():
    vals = defaultdict(lambda: defaultdict(list))
    for d in sys.argv[1:]:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(f) as fh:
                for r in csv.DictReader(fh):
                    vals[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, cs in sorted(vals.items()):
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        print(f"== {k}")
        for c in sorted(m):
            print(f"   {c:30s} {m[c]:16.1f}")
        busy = m.get("SQ_BUSY_CYCLES")
        if m.get("SQ_VALU_MFMA_BUSY_CYCLES") and busy:
            print(f"   -> MFMA busy / SQ busy cycles    {m['SQ_VALU_MFMA_BUSY_CYCLES'] / busy:8.3f} (per-SE-normalisation unknown)")
        if m.get("SQ_INSTS_MFMA") and m.get("SQ_INSTS_VALU"):
            print(f"   -> VALU insts per MFMA            {m['SQ_INSTS_VALU'] / m['SQ_INSTS_MFMA']:8.2f}")
        if m.get("SQ_WAVE_CYCLES"):
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                if c in m:
                    print(f"   -> {c} / WAVE_CYCLES   {m[c] / m['SQ_WAVE_CYCLES']:8.3f}")


if __name__ == "__main__":
    main()
