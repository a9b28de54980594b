#!/usr/bin/env python3
"""Per-channel envelope between decode/resize semantics.

The reference decodes with zune-jpeg 0.5.12 and resizes with
fast_image_resize 5.5.0, neither of which exists offline.  The product
matches the oracle's libjpeg-turbo mode (pinned to PIL) and FIR mode; this
tool measures how far those are from the oracle's restatements of the
reference's own crates (zune mode: unpinned) and from Pillow's convolution
(Pillow mode: pinned), per channel, on a seeded configs[1]-distribution
corpus (short side 128..768 so the scalar oracle finishes in seconds):

  decode:   libjpeg-turbo vs zune-jpeg restated      (decoded pixels)
  pipeline: same decode difference after crop_and_resize to 1024/32 (FIR)
  resize:   FIR (fast_image_resize restated) vs Pillow (pinned), same input

    python tools/semantics_envelope.py [--n 96] [--out profiles/r02/semantics_envelope.json]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from datago_amd import synth  # noqa: E402
from oracle import buckets as B  # noqa: E402
from oracle import oracle as O  # noqa: E402


def stats(diffs):
    """diffs: list of int arrays (H, W, C) of a - b."""
    c = max(d.shape[2] for d in diffs)
    out = {}
    for ch in range(c):
        v = np.concatenate([np.abs(d[:, :, ch]).ravel() for d in diffs if d.shape[2] > ch])
        out[f"ch{ch}"] = {"max": int(v.max()), "mean": round(float(v.mean()), 4),
                          "p99": int(np.percentile(v, 99)), "frac_nonzero": round(float((v > 0).mean()), 4)}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=96)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    datas = synth.mixed_corpus(21, a.n, 128, 768)
    t = B.ARAwareTransform(1024, 32, 0.5, 2.0)
    dec_d, dec_in, pipe_d, rs_d = [], [], [], []
    for d in datas:
        st, lj = O.jpeg_decode(d)
        with O.semantics(O.SEM_ZUNE):
            st2, zu = O.jpeg_decode(d)
        assert st == 0 and st2 == 0
        dec_d.append(lj.astype(np.int32) - zu.astype(np.int32))
        dec_in.append(dec_d[-1][:-1, :-1])  # without the last row and column (edge handling differs)
        tw, th = t.target_size(lj.shape[1], lj.shape[0])
        a_ = O.crop_and_resize(lj, tw, th, O.MODE_FIR)
        b_ = O.crop_and_resize(zu, tw, th, O.MODE_FIR)
        pipe_d.append(a_.astype(np.int32) - b_.astype(np.int32))
        p_ = O.crop_and_resize(lj, tw, th, O.MODE_PILLOW)
        rs_d.append(a_.astype(np.int32) - p_.astype(np.int32))
    res = {"corpus": f"{a.n} seeded JPEGs, configs[1] distribution (seed 21), short side 128..768",
           "decode_libjpeg_vs_zune": stats(dec_d),
           "decode_libjpeg_vs_zune_without_last_row_col": stats(dec_in),
           "pipeline_libjpeg_vs_zune_after_fir_resize_1024_32": stats(pipe_d),
           "resize_fir_vs_pillow_same_input": stats(rs_d),
           "pinning": {"libjpeg": "bit-exact vs PIL 12 / libjpeg-turbo (tests/test_oracle_jpeg.py)",
                       "zune": "UNPINNED: restated from zune-jpeg 0.5.12's published source, crate absent",
                       "fir": "UNPINNED: fast_image_resize 5.5.0 restated, crate absent",
                       "pillow": "bit-exact vs Pillow LANCZOS incl. box= crops"}}
    line = json.dumps(res, indent=1)
    print(line)
    if a.out:
        with open(a.out, "w") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()
