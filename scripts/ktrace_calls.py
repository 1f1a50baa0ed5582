"""Per-call durations (us) of kernels whose name contains a pattern, in the LAST training step of
a rocprofv3 kernel trace (steps delimited as in ktrace_steps.py), with the kernel launched
before each call. Usage: python scripts/ktrace_calls.py <kernel_trace.csv> <pattern>"""
import csv
import sys


def main():
    path, pat = sys.argv[1], sys.argv[2]
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    adam = [i for i, r in enumerate(rows) if "adam_kernel" in r[2]]
    ends = [i for j, i in enumerate(adam) if j + 1 == len(adam) or adam[j + 1] - i > 50]
    s, e = ends[-2] + 1, ends[-1]
    for i in range(s, e + 1):
        a, b, n = rows[i]
        if pat in n:
            prev = rows[i - 1][2][:60]
            nxt = rows[i + 1][2][:60] if i + 1 < len(rows) else ""
            print(f"{(b - a) / 1e3:9.1f} us  after: {prev}  | before: {nxt}")


if __name__ == "__main__":
    main()
