"""Per-kernel instruction mix of a hipcc ``-S`` listing, restricted to the hottest loop.

usage: python scripts/isa_loop_stats.py kernels.s [name-substring ...]

For every kernel whose mangled name contains all substrings, finds the basic blocks that form
backward-branch loops (a ``s_cbranch``/``s_branch`` to an earlier label) and prints the counts of
MFMA, VALU (split into transcendental / conversion / other), LDS, VMEM and SALU instructions in
the largest loop, plus VALU per MFMA. Used to check VALU-per-MFMA budgets of the attention and
GEMM kernels before spending GPU time (MI355X_MICROARCH.md: ~5 hidden fillers per 32x32x16 MFMA).
"""
import re
import sys
from collections import Counter


def kernels(path):
    name, body = None, []
    for line in open(path):
        m = re.match(r"^(_Z\S+):\s*(;.*)?$", line)
        if m:
            if name:
                yield name, body
            name, body = m.group(1), []
            continue
        if name is not None:
            if line.startswith("\t.section") or line.startswith(".Lfunc_end"):
                yield name, body
                name, body = None, []
            else:
                body.append(line.rstrip("\n"))
    if name:
        yield name, body


def classify(op):
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith(("v_exp", "v_log", "v_rcp", "v_rsq", "v_sqrt", "v_sin", "v_cos")):
        return "valu_trans"
    if op.startswith("v_cvt"):
        return "valu_cvt"
    if op.startswith(("v_cndmask", "v_cmp", "v_bfe")):
        return "valu_sel"
    if op.startswith(("v_mul_u32_u24", "v_mul_lo", "v_xor", "v_lshr", "v_lshl", "v_and", "v_or", "v_xad", "v_bfi", "v_perm")):
        return "valu_int"
    if op.startswith("v_"):
        return "valu_other"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_")):
        return "vmem"
    if op.startswith("s_"):
        return "salu"
    return "other"


def loops(body):
    labels = {}
    for i, l in enumerate(body):
        m = re.match(r"^(\.LBB\S+):", l)
        if m:
            labels[m.group(1)] = i
    out = []
    for i, l in enumerate(body):
        m = re.match(r"^\s+s_(cbranch_\w+|branch)\s+(\.LBB\S+)", l)
        if m and m.group(2) in labels and labels[m.group(2)] < i:
            out.append((labels[m.group(2)], i))
    return out


def stats(lines):
    c = Counter()
    for l in lines:
        s = l.strip()
        if not s or s.startswith((";", ".")) or s.endswith(":"):
            continue
        c[classify(s.split()[0])] += 1
    return c


def main():
    path, subs = sys.argv[1], sys.argv[2:]
    for name, body in kernels(path):
        if not all(s in name for s in subs):
            continue
        lp = loops(body)
        whole = stats(body)
        print(f"== {name[:110]}")
        print("   whole kernel:", dict(whole))
        if lp:
            a, b = max(lp, key=lambda x: stats(body[x[0]:x[1] + 1])["mfma"])
            c = stats(body[a:b + 1])
            valu = sum(v for k, v in c.items() if k.startswith("valu"))
            print(f"   hottest loop ({b - a} lines):", dict(c))
            if c["mfma"]:
                print(f"   VALU/MFMA = {valu / c['mfma']:.2f}")


if __name__ == "__main__":
    main()
