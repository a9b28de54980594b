"""GPU JPEG re-encode (pre_encode_images + encode_format jpeg) against the C
restatement of image 0.25's JpegEncoder (oracle/jpeg_enc_oracle.c): the
bytes must be identical.  The inputs go through the full decode + bucket
resize first, as in image_to_payload (image_processing.rs:341-431)."""
import io

import numpy as np
import pytest
from PIL import Image

from datago_amd import synth
from oracle import buckets as B
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _lib():
    from datago_amd import _lib as L
    return L


def _ctx(quality=92, rgb8=False, resize=True, fmt=1):
    L = _lib()
    kw = dict(pre_encode_images=True, encode_format=fmt, jpeg_quality=quality, image_to_rgb8=rgb8)
    if resize:
        kw.update(crop_and_resize=True, default_image_size=512, downsampling_ratio=16, min_aspect_ratio=0.5,
                  max_aspect_ratio=2.0)
    return L.Context(0, **kw)


def _expected(data, quality, rgb8, resize):
    st, dec = O.decode_any(data)
    assert st == 0
    h, w, c = dec.shape
    resized = False
    if resize:
        tw, th = B.ARAwareTransform(512, 16, 0.5, 2.0).target_size(w, h)
        if (tw, th) != (w, h):
            dec = O.crop_and_resize(dec, tw, th, O.MODE_FIR)
            resized = True
    if rgb8:
        dec = O.to_rgb8(dec, resized)
    elif dec.shape[2] == 2 and resized:  # GrayImage over the LA bytes
        hh, ww = dec.shape[:2]
        dec = np.ascontiguousarray(dec).reshape(-1)[: ww * hh].reshape(hh, ww, 1)
    return O.jpeg_encode(dec, quality), dec


def _inputs():
    rng = np.random.default_rng(5)
    out = []
    for i in range(10):
        w, h = int(rng.integers(8, 700)), int(rng.integers(8, 700))
        out.append(synth.make_jpeg(100 + i, w, h, 90, ["4:2:0", "4:4:4", "4:2:2"][i % 3], gray=(i == 4)))
    for i, kind in enumerate(["RGB", "L", "RGBA", "LA", "P8"]):
        out.append(synth.make_png(200 + i, 150 + 40 * i, 120 + 17 * i, kind))
    out.append(synth.make_jpeg(300, 1, 1, 90))
    out.append(synth.make_jpeg(301, 592, 432, 90))  # exact bucket size: no resize
    return out


@pytest.mark.parametrize("quality,rgb8,resize", [(92, False, True), (92, True, True), (50, False, False),
                                                 (100, True, False), (75, False, True)])
def test_encode_bit_exact_vs_oracle(quality, rgb8, resize):
    ctx = _ctx(quality, rgb8, resize)
    datas = _inputs()
    res = ctx.decode_batch(datas)
    for d, (st, enc, m) in zip(datas, res):
        assert st == 0, _lib().last_error()
        exp, img = _expected(d, quality, rgb8, resize)
        assert m.is_encoded == 1 and m.channels == -1
        assert (m.width, m.height) == (img.shape[1], img.shape[0])
        assert enc.tobytes() == exp, (len(enc), len(exp))
        im = Image.open(io.BytesIO(enc.tobytes()))
        assert im.size == (img.shape[1], img.shape[0])


def test_encode_round_trip_quality():
    ctx = _ctx(92, False, True)
    d = synth.make_jpeg(7, 900, 700, 95, "4:4:4")
    (st, enc, m), = ctx.decode_batch([d])
    assert st == 0
    _, img = _expected(d, 92, False, True)
    back = np.asarray(Image.open(io.BytesIO(enc.tobytes()))).astype(np.float64)
    psnr = 10 * np.log10(255 ** 2 / ((back - img) ** 2).mean())
    assert psnr > 30


def test_png_reencode_unsupported():
    L = _lib()
    ctx = _ctx(92, False, True, fmt=0)
    (st, _, _), = ctx.decode_batch([synth.make_jpeg(8, 64, 64, 90)])
    assert st == L.DG_ERR_UNSUPPORTED
