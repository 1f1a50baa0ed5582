"""Per-kernel VGPR/AGPR/spill/occupancy summary for one HIP source (gfx950).

Usage: python scripts/kres.py smdt_amd/csrc/kernels/flash_attn.hip
"""
import re
import subprocess
import sys

src = sys.argv[1]
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-I", "smdt_amd/csrc", "-c", src,
       "-o", "/tmp/_kres.o", "-Rpass-analysis=kernel-resource-usage"]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
cur = None
rows = {}
for line in out.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = m.group(1)
        rows[cur] = {}
        continue
    m = re.search(r"remark: ([A-Za-z ]+?)(?: \[waves/SIMD\])?: (\d+)", line)
    if m and cur:
        rows[cur][m.group(1).strip()] = int(m.group(2))
for k, v in rows.items():
    dem = subprocess.run(["c++filt", k], capture_output=True, text=True).stdout.strip()
    dem = re.sub(r"\(.*", "", dem)[:70]
    print(f"{dem:72s} vgpr {v.get('VGPRs', 0):3d} agpr {v.get('AGPRs', 0):3d} "
          f"spill {v.get('VGPRs Spill', 0):3d} occ {v.get('Occupancy', 0)} lds {v.get('LDS Size', 0)}")
