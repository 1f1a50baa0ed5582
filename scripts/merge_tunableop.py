"""Merge TunableOp result CSVs: rows of the later files replace the earlier ones' rows for the
same (op, shape) key; validator lines come from the first file.
Usage: python scripts/merge_tunableop.py out.csv base.csv new1.csv [new2.csv ...]"""
import sys


def main():
    out, files = sys.argv[1], sys.argv[2:]
    header, rows = [], {}
    for i, f in enumerate(files):
        for line in open(f):
            line = line.rstrip("\n")
            if not line:
                continue
            parts = line.split(",")
            if parts[0] == "Validator":
                if i == 0:
                    header.append(line)
                continue
            rows[(parts[0], parts[1])] = line
    with open(out, "w") as fo:
        fo.write("\n".join(header + list(rows.values())) + "\n")
    print(f"{len(rows)} tuned shapes -> {out}")


if __name__ == "__main__":
    main()
