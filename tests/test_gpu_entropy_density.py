"""Per-image subsequence size (context option "sub_density"): images with few
coded bits per block decode in shorter entropy ranges (half / a quarter of
the batch's size) with their own checkpoint records.  Bit-exact against the
oracle and the uniform sizing, on flat low-quality images (the ones that get
the short ranges), detailed ones, restart markers, gray and all samplings."""
import numpy as np
import pytest

from datago_amd import synth
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _flat(seed, w, h, q, ss):
    yy, xx = np.mgrid[0:h, 0:w]
    arr = np.stack([(xx * 255 // max(w - 1, 1)), (yy * 255 // max(h - 1, 1)), ((xx + yy + seed) % 256)], -1)
    return synth.encode_jpeg(arr.astype(np.uint8), q, ss)


def test_sub_density_bit_exact():
    from datago_amd import _lib as L
    datas = [_flat(i, 900 + 37 * i, 700 - 23 * i, [10, 20, 30][i % 3], ["4:2:0", "4:2:2", "4:4:4"][i % 3])
             for i in range(6)]
    datas += [synth.make_jpeg(8300 + i, 800, 600, q, ss, restart_marker_rows=r, gray=g)
              for i, (q, ss, r, g) in enumerate([(95, "4:2:0", 0, False), (40, "4:2:0", 1, False),
                                                  (70, "4:4:4", 0, True), (15, "4:2:2", 2, False)])]
    ref_ctx, ctx = L.Context(0), L.Context(0)
    for c in (ref_ctx, ctx):
        c.set_option("sub_bits", 0)
    ctx.set_option("sub_density", 64)
    a, b = ctx.decode_batch(datas), ref_ctx.decode_batch(datas)
    for i, (d, (st, x, _), (st2, y, _)) in enumerate(zip(datas, a, b)):
        assert st == 0 and st2 == 0, i
        assert np.array_equal(x, y), i
        assert np.array_equal(x.reshape(O.jpeg_decode(d)[1].shape), O.jpeg_decode(d)[1]), i
