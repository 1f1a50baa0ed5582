"""Plot an Oxford run's ``model_history.p`` (JSON of per-epoch lists) — the reference notebook's
result-analysis cells (SURVEY R16, NB2:3383-3505). Accepts the history file or a ``model.tar.gz``.

usage: python scripts/plot_history.py model.tar.gz --out curves.png
"""
import argparse
import json
import os
import tarfile


def load_history(path: str):
    if path.endswith((".tar.gz", ".tgz")):
        with tarfile.open(path) as t:
            m = next(x for x in t.getmembers() if os.path.basename(x.name) == "model_history.p")
            return json.loads(t.extractfile(m).read().decode())
    with open(path) as f:
        return json.load(f)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("history")
    p.add_argument("--out", default="history.png")
    a = p.parse_args()
    h = load_history(a.history)
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    # keys written by recipes/2_training_oxford-pet_ddp/util.py (per-batch train, per-epoch val avg)
    panels = [("loss", ["losses", "val_avg_losses"]), ("top1", ["top1", "val_avg_top1"]),
              ("top5", ["top5", "val_avg_top5"])]
    fig, axes = plt.subplots(1, 3, figsize=(15, 4))
    for ax, (title, keys) in zip(axes, panels):
        for k in keys:
            if k in h and h[k]:
                ax.plot(range(1, len(h[k]) + 1), h[k], label=k)
        ax.set_title(title)
        ax.set_xlabel("logged step / epoch")
        ax.legend()
    fig.tight_layout()
    fig.savefig(a.out)
    print(f"wrote {a.out}: " + ", ".join(f"{k}[{len(v)}]" for k, v in h.items() if isinstance(v, list)))


if __name__ == "__main__":
    main()
