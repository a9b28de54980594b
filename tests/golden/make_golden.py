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

Usage: python tests/golden/make_golden.py
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


def main():
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
