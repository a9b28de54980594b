"""GPU debug: bisect the resize path (coeff stream / resize-H staging) against the oracle."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from datago_amd import _lib, synth
from oracle import oracle as O, buckets as B
data = synth.make_jpeg(1, 640, 480, 90, "4:2:0")
st, dec = O.jpeg_decode(data)
nw, nh = B.scaled_size(640, 480, 592, 432)
r1 = O.resample(dec, nw, nh, (0, 0, 640, 480))
l, t, cw, ch = B.fit_crop_box(nw, nh, 592, 432)
r2 = O.resample(r1, 592, 432, (l, t, l + cw, t + ch))
for side in (1, 0):
    for dbg in (0, 1):
        ctx = _lib.Context(0, crop_and_resize=True, default_image_size=512, downsampling_ratio=16,
                           min_aspect_ratio=0.5, max_aspect_ratio=2.0)
        ctx.set_option("side_stream", side)
        ctx.set_option("debug_flags", dbg)
        s, arr, meta = ctx.decode_one(data)
        d = np.abs(arr.astype(int) - r2.astype(int))
        bad = np.argwhere(d.max(axis=2) > 0)
        print(f"side={side} nostage={dbg}: status={s} maxdiff={d.max()} ndiff={int((d>0).sum())} "
              f"first bad={bad[:5].tolist()} rows_bad={len(set(bad[:,0].tolist())) if len(bad) else 0} "
              f"cols_bad={len(set(bad[:,1].tolist())) if len(bad) else 0}")
        if len(bad):
            y, x = bad[0]
            print("   gpu", arr[y, x:x+4].tolist(), "ref", r2[y, x:x+4].tolist())
