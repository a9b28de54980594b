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


def _png_check(data: bytes):
    """Container checks independent of PIL: chunk CRCs, zlib stream, Adler-32."""
    import binascii
    import struct
    import zlib
    assert data[:8] == b"\x89PNG\r\n\x1a\n"
    pos, idat, types = 8, b"", []
    while pos < len(data):
        n, = struct.unpack(">I", data[pos:pos + 4])
        t = data[pos + 4:pos + 8]
        body = data[pos + 8:pos + 8 + n]
        crc, = struct.unpack(">I", data[pos + 8 + n:pos + 12 + n])
        assert binascii.crc32(t + body) & 0xFFFFFFFF == crc, t
        types.append(t)
        if t == b"IDAT":
            idat += body
        pos += 12 + n
    assert types[0] == b"IHDR" and types[-1] == b"IEND" and pos == len(data)
    return zlib.decompress(idat)  # checks the Adler-32


@pytest.mark.parametrize("rgb8", [False, True])
def test_png_reencode_lossless(rgb8):
    """pre_encode_images + encode_format png (image_processing.rs:396-413):
    the GPU's PNG (adaptive filters, fixed-Huffman DEFLATE with run matches)
    must decode -- with PIL, zlib and the oracle -- to exactly the image the
    same context computes without encoding.  The bytes are not the png
    crate's (fdeflate is not vendored): parity is on the pixels."""
    L = _lib()
    kw = dict(crop_and_resize=True, default_image_size=512, downsampling_ratio=16, min_aspect_ratio=0.5,
              max_aspect_ratio=2.0, image_to_rgb8=rgb8)
    enc = L.Context(0, pre_encode_images=True, encode_format=0, **kw)
    raw = L.Context(0, **kw)
    datas = [synth.make_jpeg(30, 640, 480, 90), synth.make_jpeg(31, 300, 700, 85, gray=True),
             synth.make_png(32, 512, 512, "RGBA"), synth.make_png(33, 200, 150, "LA"),
             synth.make_png(34, 333, 444, "L"), synth.make_png(35, 700, 300, "P8T"),
             synth.make_png(36, 1, 1, "RGB"), synth.make_png(37, 512, 512, "LA")]
    # a flat mask: long runs compress through the distance-1 matches
    m = np.zeros((600, 800), np.uint8)
    m[100:400, 200:650] = 255
    datas.append(synth.pil_png(m))
    er, rr = enc.decode_batch(datas), raw.decode_batch(datas)
    for i, (d, (se, pe, me), (sr, pr, mr)) in enumerate(zip(datas, er, rr)):
        assert se == 0 and sr == 0, (i, se, sr, L.last_error())
        assert me.is_encoded == 1 and me.channels == -1 and me.nbytes == len(pe.tobytes())
        png = pe.tobytes()
        filt = _png_check(png)
        st, dec = O.png_decode(png)
        assert st == 0
        ref = pr.reshape(mr.height, mr.width, -1)
        if ref.shape[2] == 2 and (mr.original_width, mr.original_height) != (mr.width, mr.height):
            # resized LA: a GrayImage over the first w*h LA bytes
            ref = ref.reshape(-1)[: mr.width * mr.height].reshape(mr.height, mr.width, 1)
        assert dec.shape == ref.shape and np.array_equal(dec, ref), i
        pil = np.asarray(Image.open(io.BytesIO(png)))
        assert np.array_equal(pil.reshape(ref.shape), ref), i
        assert len(filt) == ref.shape[0] * (ref.shape[1] * ref.shape[2] + 1)
    # the flat mask compresses well
    assert er[-1][2].nbytes < 0.05 * 800 * 600
