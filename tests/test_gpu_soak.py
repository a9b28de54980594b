"""Mixed-batch soak: random JPEGs (baseline, restart intervals, gray, every
subsampling and quality) and PNGs (every kind, Adam7) of random sizes in ONE
batch per configuration (bucket tables 224/16, 512/16, 1024/32; RGB8
conversion on and off), each output checked bit for bit against the oracle's
decode -> crop_and_resize -> convert_to_rgb8.  What the per-feature suites do
not cover: descriptor indexing, list ordering and buffer layout with every
format interleaved in one launch set."""
import numpy as np
import pytest

from datago_amd import synth
from oracle import buckets as B
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _lib():
    from datago_amd import _lib as L
    return L


def _corpus(seed: int, n: int):
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        w, h = int(rng.integers(1, 1500)), int(rng.integers(1, 1500))
        if rng.random() < 0.6:
            out.append(synth.make_jpeg(seed * 1000 + i, w, h, int(rng.integers(30, 101)),
                                       ["4:2:0", "4:2:2", "4:4:4"][int(rng.integers(0, 3))], bool(rng.random() < 0.1),
                                       restart_marker_rows=int(rng.integers(0, 4)) if rng.random() < 0.3 else 0))
        else:
            out.append(synth.make_png(seed * 1000 + i, min(w, 900), min(h, 900),
                                      synth.PNG_KINDS[int(rng.integers(0, len(synth.PNG_KINDS)))],
                                      interlace=bool(rng.random() < 0.2)))
    return out


@pytest.mark.parametrize("cfg", [(224, 16, False), (512, 16, True), (1024, 32, False)],
                         ids=lambda c: f"{c[0]}-{c[1]}-{'rgb8' if c[2] else 'raw'}")
def test_mixed_batch_soak(cfg):
    size, ratio, rgb8 = cfg
    L = _lib()
    ctx = L.Context(0, crop_and_resize=True, default_image_size=size, downsampling_ratio=ratio,
                    min_aspect_ratio=0.5, max_aspect_ratio=2.0, image_to_rgb8=rgb8)
    datas = _corpus(size + ratio, 48)
    t = B.ARAwareTransform(size, ratio, 0.5, 2.0)
    for i, (d, (st, arr, meta)) in enumerate(zip(datas, ctx.decode_batch(datas))):
        assert st == 0, (i, L.last_error())
        ost, dec = O.decode_any(d)
        assert ost == 0
        if dec.ndim == 2:
            dec = dec[:, :, None]
        h, w = dec.shape[:2]
        tw, th = t.target_size(w, h)
        ref = O.crop_and_resize(dec, tw, th, O.MODE_FIR) if (w, h) != (tw, th) else dec
        if rgb8:
            ref = O.to_rgb8(ref, (w, h) != (tw, th))
        assert arr.reshape(ref.shape).shape == ref.shape and np.array_equal(arr.reshape(ref.shape), ref), (i, w, h)
