"""Per-channel max |GPU - oracle| of the golden JPEGs at 512/16 buckets under
context-option variants (debug probe for bit-exactness regressions)."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from datago_amd import _lib as L  # noqa: E402
from oracle import buckets as B  # noqa: E402
from oracle import oracle as O  # noqa: E402

GOLD = os.path.join(ROOT, "tests", "golden")
names = sorted(json.load(open(os.path.join(GOLD, "jpeg_expected.json"))).keys())
files = [(n, open(os.path.join(GOLD, "jpeg", n + ".jpg"), "rb").read()) for n in names]
t = B.ARAwareTransform(512, 16, 0.5, 2.0)
variants = [{}, {"h_pairs": 0}, {"chroma_rec": 0}, {"h_pairs": 0, "chroma_rec": 0}]
for sem in (0, 1):
    for var in variants:
        ctx = L.Context(0, crop_and_resize=True, default_image_size=512, downsampling_ratio=16,
                        min_aspect_ratio=0.5, max_aspect_ratio=2.0, decode_semantics=sem)
        for k, v in var.items():
            ctx.set_option(k, v)
        bad = []
        for (name, data), (st, arr, meta) in zip(files, ctx.decode_batch([d for _, d in files])):
            with O.semantics(sem):
                dec = O.jpeg_decode(data)[1]
            ref = O.crop_and_resize(dec, *t.target_size(dec.shape[1], dec.shape[0]), O.MODE_FIR)
            if st or arr.shape != ref.shape:
                bad.append((name, "status", st))
                continue
            d = np.abs(arr.astype(int) - ref.astype(int)).reshape(-1, arr.shape[2]).max(axis=0)
            if d.max():
                bad.append((name, d.tolist()))
        print("sem", sem, var, "bad:", bad, flush=True)
        ctx.close()
