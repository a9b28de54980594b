"""Generate the committed golden fixtures (run here, in the build container).

* tests/golden/jpeg/*.jpg   — small seeded JPEGs (PIL/libjpeg-turbo 3.1 encoder)
* tests/golden/jpeg_expected.json — sha256 + shape of PIL's decode of each file
  (PIL = libjpeg-turbo ISLOW IDCT + fancy upsampling: the oracle's target)
* tests/golden/resize_expected.json — sha256 of Pillow's two-step
  resize(LANCZOS) + resize(LANCZOS, box=fit-crop) of each decode into its
  bucket (the structure the oracle's MODE_PILLOW must reproduce exactly)
* tests/golden/buckets.json — bucket tables + closest-bucket answers for the
  BASELINE configs, from oracle/buckets.py (itself pinned by the reference's
  known answers at image_processing.rs:441-478).

* tests/golden/png/*.png    — small seeded PNGs (every colour type, sub-byte
  depths, palettes with tRNS, all five filters, stored / fixed / dynamic
  blocks, split IDAT chunks, PIL's own encoder) plus 16-bit / interlaced /
  corrupt files
* tests/golden/png_expected.json — status + sha256 + shape of PIL's decode of
  each (expanded like png's Transformations::EXPAND)

Usage: python tests/golden/make_golden.py [--png-only]
"""
import hashlib
import io
import json
import os
import sys

import numpy as np
from PIL import Image

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from datago_amd import synth  # noqa: E402
from oracle import buckets as B  # noqa: E402

CASES = [
    # name, w, h, quality, subsampling, gray, restart_rows
    ("1x1_420", 1, 1, 90, "4:2:0", False, 0),
    ("3x3_422", 3, 3, 90, "4:2:2", False, 0),
    ("4x4_420", 4, 4, 75, "4:2:0", False, 0),
    ("5x7_444", 5, 7, 95, "4:4:4", False, 0),
    ("17x13_420", 17, 13, 90, "4:2:0", False, 0),
    ("33x31_422", 33, 31, 85, "4:2:2", False, 0),
    ("64x48_gray", 64, 48, 90, "4:2:0", True, 0),
    ("100x75_444", 100, 75, 100, "4:4:4", False, 0),
    ("123x457_420", 123, 457, 60, "4:2:0", False, 0),
    ("1000x10_420", 1000, 10, 90, "4:2:0", False, 0),
    ("10x1000_420", 10, 1000, 90, "4:2:0", False, 0),
    ("640x480_420", 640, 480, 90, "4:2:0", False, 0),
    ("640x480_420_rst1", 640, 480, 90, "4:2:0", False, 1),
    ("301x199_gray_rst2", 301, 199, 80, "4:2:0", True, 2),
    ("517x389_422_rst3", 517, 389, 92, "4:2:2", False, 3),
    ("250x600_444_q30", 250, 600, 30, "4:4:4", False, 0),
]


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


PNG_CASES = [
    # name, kind, w, h, encoder kwargs
    ("rgb_17x9_dyn", "RGB", 17, 9, {}),
    ("rgba_33x20_dyn", "RGBA", 33, 20, {}),
    ("l_64x33_paeth", "L", 64, 33, {"filters": "4"}),
    ("la_31x17_avg", "LA", 31, 17, {"filters": "3"}),
    ("p8_40x30_stored", "P8", 40, 30, {"level": 0}),
    ("p8t_25x25_fixed", "P8T", 25, 25, {"strategy": 4}),
    ("p4_19x7_split", "P4", 19, 7, {"idat_max": 5}),
    ("p2_13x11", "P2", 13, 11, {}),
    ("p1_70x3", "P1", 70, 3, {}),
    ("l1_9x9", "L1", 9, 9, {}),
    ("l2_21x5", "L2", 21, 5, {}),
    ("l4_11x13", "L4", 11, 13, {}),
    ("lt_15x15", "LT", 15, 15, {}),
    ("rgbt_12x10", "RGBT", 12, 10, {}),
    ("rgb_1x1", "RGB", 1, 1, {}),
    ("rgb_300x200_l9", "RGB", 300, 200, {"level": 9}),
]


def png_golden():
    import zlib
    os.makedirs(os.path.join(HERE, "png"), exist_ok=True)
    exp = {}

    def pil_expand(data):
        im = Image.open(io.BytesIO(data))
        trns = "transparency" in im.info
        if im.mode == "P":
            im = im.convert("RGBA" if trns else "RGB")
        elif im.mode in ("1", "L"):
            im = im.convert("LA" if trns else "L")
        elif im.mode == "RGB" and trns:
            im = im.convert("RGBA")
        a = np.asarray(im)
        return a[:, :, None] if a.ndim == 2 else a

    files = {}
    for i, (name, kind, w, h, kw) in enumerate(PNG_CASES):
        files[name] = synth.make_png(2000 + i, w, h, kind, **kw)
    rng = np.random.default_rng(7)
    files["pil_rgb_97x61"] = synth.pil_png(synth.synth_pixels(rng, 97, 61))
    files["pil_rgba_50x40_opt"] = synth.pil_png(
        np.concatenate([synth.synth_pixels(rng, 50, 40), rng.integers(0, 256, (40, 50, 1), dtype=np.uint8)], 2),
        optimize=True)
    rows = rng.integers(0, 256, (5, 16), dtype=np.uint8)
    files["l16_8x5_unsupported"] = synth.encode_png(rows, 8, 5, 16, 0, 2, rng)
    # Adam7-interlaced (PNG spec 8.2), expected pixels from PIL
    files["rgb_40x30_adam7"] = synth.make_png(2100, 40, 30, "RGB", interlace=True)
    files["p2_13x11_adam7"] = synth.make_png(2101, 13, 11, "P2", interlace=True)
    files["la_5x3_adam7"] = synth.make_png(2102, 5, 3, "LA", interlace=True)
    good = files["rgb_17x9_dyn"]
    files["truncated_corrupt"] = good[: len(good) - 30]
    for name, data in files.items():
        with open(os.path.join(HERE, "png", name + ".png"), "wb") as f:
            f.write(data)
        if name.endswith("_unsupported"):
            exp[name] = {"status": 1}
            continue
        if name.endswith("_corrupt"):
            exp[name] = {"status": 2}
            continue
        a = pil_expand(data)
        exp[name] = {"status": 0, "shape": list(a.shape), "sha256": sha(a)}
    with open(os.path.join(HERE, "png_expected.json"), "w") as f:
        json.dump(exp, f, indent=1, sort_keys=True)
    print("wrote", len(files), "png fixtures")


def main():
    png_golden()
    if "--png-only" in sys.argv:
        return
    jexp, rexp = {}, {}
    tr = B.ARAwareTransform(512, 16, 0.5, 2.0)
    for i, (name, w, h, q, ss, gray, rst) in enumerate(CASES):
        data = synth.make_jpeg(1000 + i, w, h, q, ss, gray, rst)
        with open(os.path.join(HERE, "jpeg", name + ".jpg"), "wb") as f:
            f.write(data)
        im = Image.open(io.BytesIO(data))
        arr = np.asarray(im)
        jexp[name] = {"shape": list(arr.shape), "sha256": sha(arr), "mode": im.mode}
        tw, th = tr.target_size(w, h)
        if (w, h) == (tw, th):
            out = arr
        else:
            nw, nh = B.scaled_size(w, h, tw, th)
            l, t, cw, ch = B.fit_crop_box(nw, nh, tw, th)
            out = np.asarray(im.resize((nw, nh), Image.LANCZOS)
                             .resize((tw, th), Image.LANCZOS, box=(l, t, l + cw, t + ch)))
        rexp[name] = {"bucket": [tw, th], "shape": list(out.shape), "sha256": sha(out),
                      "config": "512/16/0.5/2.0"}
    with open(os.path.join(HERE, "jpeg_expected.json"), "w") as f:
        json.dump(jexp, f, indent=1, sort_keys=True)
    with open(os.path.join(HERE, "resize_expected.json"), "w") as f:
        json.dump(rexp, f, indent=1, sort_keys=True)

    bk = {}
    grid = [(w, h) for w in (1, 7, 100, 224, 300, 400, 480, 500, 640, 1000, 1024, 1920, 4000)
            for h in (1, 9, 100, 200, 333, 375, 480, 640, 768, 1000, 1080, 3000)]
    for cfg, (size, ratio, lo, hi) in B.CONFIGS.items():
        t = B.ARAwareTransform(size, ratio, lo, hi)
        bk[cfg] = {
            "params": [size, ratio, lo, hi],
            "size_list": B.build_image_size_list(size, ratio, lo, hi),
            "keys": [k for _, k in t.aspect_ratios],
            "sizes": [t.aspect_ratio_to_size[k] for _, k in t.aspect_ratios],
            "closest": [[w, h, t.get_closest_aspect_ratio(w, h)] for (w, h) in grid],
        }
    with open(os.path.join(HERE, "buckets.json"), "w") as f:
        json.dump(bk, f, indent=1)
    print("wrote", len(CASES), "jpeg fixtures")


if __name__ == "__main__":
    main()
