"""Per-kernel averages of a pmc_gemm.sh run (gemm_tn vs the library GEMM): python
scripts/pmc_gemm_summary.py <dir with p1/ p2/> [out.json]"""
import collections
import csv
import json
import sys

base = sys.argv[1]
out = {}
for p in ("p1", "p2"):
    rows = list(csv.DictReader(open(f"{base}/{p}/run_counter_collection.csv")))
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    meta = {}
    for r in rows:
        k = r["Kernel_Name"]
        if "gemm_tn_kernel" not in k and "Cijk" not in k:
            continue
        if "Cijk" in k:
            k = "library " + k.split("_UserArgs")[0][-40:]
        else:
            k = "gemm_tn " + k[:60]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r["Dispatch_Id"])
        meta[k] = {"wg": r["Workgroup_Size"], "lds": r["LDS_Block_Size"], "vgpr": r["VGPR_Count"]}
    for k, v in agg.items():
        d = out.setdefault(k, dict(meta[k]))
        d.update({c: round(x / len(disp[k])) for c, x in v.items()})
for k, d in out.items():
    if "TCC_HIT_sum" in d:
        d["tcc_requests"] = d["TCC_HIT_sum"] + d["TCC_MISS_sum"]
print(json.dumps(out, indent=1))
if len(sys.argv) > 2:
    json.dump(out, open(sys.argv[2], "w"), indent=1)
