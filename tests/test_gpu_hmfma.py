"""k_resize_hm: the band H passes (fast_image_resize's horizontal convolution,
image_processing.rs:288-323, both resize calls) on the i8 matrix cores.
Tolerance 0: bit-exact against the oracle and against the VALU band kernel
(option h_mfma = 0) for colour JPEGs (fused upsampling + colour fill), gray
JPEGs and PNGs of 1-4 channels (byte fill, alpha premultiplied around the
passes), upscales and downscales in both K-step classes, x.5 crops (the
call-2 H pass), and both JPEG decode semantics."""
import numpy as np
import pytest

from datago_amd import synth
from oracle import buckets as B
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _ctx(size, ratio, mfma, sem=0):
    from datago_amd import _lib as L
    c = L.Context(0, crop_and_resize=True, default_image_size=size, downsampling_ratio=ratio, min_aspect_ratio=0.5,
                  max_aspect_ratio=2.0, decode_semantics=sem)
    c.set_option("h_mfma", mfma)
    return c


@pytest.mark.parametrize("size,ratio,sem", [(1024, 32, 0), (512, 16, 1)])
def test_h_mfma_jpeg_bit_exact(size, ratio, sem):
    tr = B.ARAwareTransform(size, ratio, 0.5, 2.0)
    datas = []
    for i, (w, h) in enumerate([(300, 200), (640, 480), (1100, 830), (2100, 1500), (3300, 2400), (4400, 1900),
                                (1900, 4400), (33, 17), (1300, 16), (597, 448), (2047, 1023), (777, 1555)]):
        datas.append(synth.make_jpeg(8100 + i, w, h, 60 + 3 * i, ["4:2:0", "4:2:2", "4:4:4"][i % 3], gray=i % 5 == 4))
    a, b = _ctx(size, ratio, 1, sem).decode_batch(datas), _ctx(size, ratio, 0, sem).decode_batch(datas)
    for i, (d, (st, x, _), (st2, y, _)) in enumerate(zip(datas, a, b)):
        assert st == 0 and st2 == 0, i
        assert np.array_equal(x, y), i
        with O.semantics(sem):
            _, dec = O.jpeg_decode(d)
        assert np.array_equal(x, O.crop_and_resize(dec, *tr.target_size(dec.shape[1], dec.shape[0]), O.MODE_FIR)), i


def test_h_mfma_png_channels_bit_exact():
    tr = B.ARAwareTransform(512, 16, 0.5, 2.0)
    datas = [synth.make_png(8200 + i, w, h, kind) for i, (kind, w, h) in enumerate(
        [("L", 700, 300), ("LA", 300, 700), ("RGB", 900, 650), ("RGBA", 650, 900), ("P8T", 400, 300), ("RGBA", 40, 70)])]
    a, b = _ctx(512, 16, 1).decode_batch(datas), _ctx(512, 16, 0).decode_batch(datas)
    for i, (d, (st, x, _), (st2, y, _)) in enumerate(zip(datas, a, b)):
        assert st == 0 and st2 == 0, i
        assert np.array_equal(x, y), i
        _, dec = O.png_decode(d)
        assert np.array_equal(x.reshape(-1), O.crop_and_resize(dec, *tr.target_size(dec.shape[1], dec.shape[0]),
                                                               O.MODE_FIR).reshape(-1)), i
