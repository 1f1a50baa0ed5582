"""Oxford-IIIT Pet preparation (the reference notebook's data-prep cells; NB2).

From an extracted ``images/`` directory (``<Breed_Name>_<id>.jpg`` files):
  1. drop files that are not decodable JPEGs (full decode + the JPEG end-of-image marker FFD9),
  2. bucket by breed (file name minus the trailing ``_<id>``),
  3. split into ``train/`` and ``test/`` class folders (ImageFolder layout) with a fixed seed.

No network: point it at a local copy. ``--synthetic N`` writes an N-image stand-in instead.
usage: python scripts/prepare_oxford_pet.py --images images/ --out data/oxford --test-ratio 0.2
"""
import argparse
import os
import random
import shutil
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def is_valid_jpeg(path: str) -> bool:
    try:
        with open(path, "rb") as f:
            data = f.read()
        if len(data) < 4 or data[:2] != b"\xff\xd8" or data.rstrip(b"\x00")[-2:] != b"\xff\xd9":
            return False
        from PIL import Image
        with Image.open(path) as im:
            im.convert("RGB").load()
        return True
    except Exception:
        return False


def breed_of(fname: str) -> str:
    stem = os.path.splitext(fname)[0]
    return stem.rsplit("_", 1)[0]


def prepare(images: str, out: str, test_ratio: float = 0.2, seed: int = 42, link: bool = False):
    files = sorted(f for f in os.listdir(images) if f.lower().endswith((".jpg", ".jpeg")))
    good, bad = [], []
    for f in files:
        (good if is_valid_jpeg(os.path.join(images, f)) else bad).append(f)
    by = {}
    for f in good:
        by.setdefault(breed_of(f), []).append(f)
    rng = random.Random(seed)
    counts = {"train": 0, "test": 0}
    for breed, fs in sorted(by.items()):
        fs = sorted(fs)
        rng.shuffle(fs)
        nt = max(1, int(round(len(fs) * test_ratio))) if len(fs) > 1 else 0
        for split, sel in (("test", fs[:nt]), ("train", fs[nt:])):
            d = os.path.join(out, split, breed)
            os.makedirs(d, exist_ok=True)
            for f in sel:
                src, dst = os.path.join(images, f), os.path.join(d, f)
                if link:
                    if not os.path.exists(dst):
                        os.symlink(os.path.abspath(src), dst)
                else:
                    shutil.copyfile(src, dst)
                counts[split] += 1
    return {"classes": len(by), "dropped": bad, **counts}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--images")
    p.add_argument("--out", required=True)
    p.add_argument("--test-ratio", type=float, default=0.2)
    p.add_argument("--seed", type=int, default=42)
    p.add_argument("--link", action="store_true", help="symlink instead of copying")
    p.add_argument("--synthetic", type=int, default=0)
    a = p.parse_args()
    if a.synthetic:
        from smdt_amd.data.image_folder import write_synthetic_image_folder
        write_synthetic_image_folder(a.out, num_classes=37, per_class=max(1, a.synthetic // 37))
        print(f"wrote a synthetic 37-class ImageFolder under {a.out}")
        return
    r = prepare(a.images, a.out, a.test_ratio, a.seed, a.link)
    print(f"{r['classes']} breeds, train {r['train']}, test {r['test']}, dropped {len(r['dropped'])} bad files")


if __name__ == "__main__":
    main()
