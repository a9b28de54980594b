"""k_band_dec bring-up: where does the fused path differ from the split path
(option band_dec 0)?  Prints, per image, the differing pixels' count, max,
channels and their row/column patterns."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from datago_amd import _lib as L  # noqa: E402
from datago_amd import synth  # noqa: E402


def ctx(band, size=1024, ratio=32):
    c = L.Context(0, crop_and_resize=True, default_image_size=size, downsampling_ratio=ratio, min_aspect_ratio=0.5,
                  max_aspect_ratio=2.0)
    c.set_option("band_dec", band)
    return c


cases = [(417, 768, "4:2:0", False), (640, 480, "4:4:4", False), (640, 480, "4:2:2", False), (640, 480, "4:2:0", False),
         (640, 480, "4:2:0", True), (1500, 1000, "4:2:0", False), (300, 200, "4:4:4", False), (2000, 1300, "4:4:4", True)]
datas = [synth.make_jpeg(9000 + i, w, h, 85, ss, gray=g) for i, (w, h, ss, g) in enumerate(cases)]
a, b = ctx(1).decode_batch(datas), ctx(0).decode_batch(datas)
for (w, h, ss, g), (st, x, m), (st2, y, _) in zip(cases, a, b):
    d = np.abs(x.astype(int) - y.astype(int))
    if d.ndim == 2:
        d = d[:, :, None]
    nz = np.argwhere(d.max(axis=2) > 0)
    print(f"{w}x{h} {ss} gray={g} -> {x.shape} status {st},{st2}: differ {len(nz)} / {d.shape[0] * d.shape[1]} px, "
          f"max {d.max()}, per channel {[int((d[:, :, c] > 0).sum()) for c in range(d.shape[2])]}")
    if len(nz):
        rows, cols = nz[:, 0], nz[:, 1]
        print("   rows", rows.min(), rows.max(), "row%16 hist", np.bincount(rows % 16, minlength=16).tolist())
        print("   cols", cols.min(), cols.max(), "col%16 hist", np.bincount(cols % 16, minlength=16).tolist())
        print("   first", nz[:8].tolist())
