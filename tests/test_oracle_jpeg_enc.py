"""Pin the C restatement of image 0.25's JpegEncoder (oracle/jpeg_enc_oracle.c):
quantisation tables against libjpeg's quality scaling (PIL), Huffman tables
against the DHT segments libjpeg writes (standard Annex K tables), and the
codec as a whole by round trips through PIL's decoder.  The crate's exact
byte stream is unpinned (the crate is not present offline)."""
import io
import struct

import numpy as np
import pytest
from PIL import Image

from datago_amd import synth
from oracle import oracle as O


def _segments(data: bytes):
    i, out = 2, []
    while i + 4 <= len(data):
        assert data[i] == 0xFF
        m = data[i + 1]
        n = struct.unpack(">H", data[i + 2:i + 4])[0]
        out.append((m, data[i + 4:i + 2 + n]))
        if m == 0xDA:
            break
        i += 2 + n
    return out


@pytest.mark.parametrize("q", [1, 10, 50, 75, 92, 100])
def test_quant_tables_match_libjpeg(q):
    buf = io.BytesIO()
    Image.fromarray(np.zeros((8, 8, 3), np.uint8)).save(buf, "JPEG", quality=q, subsampling=0)
    pq = Image.open(io.BytesIO(buf.getvalue())).quantization  # natural order (Pillow >= 8)
    ours = O.jpeg_qtables(q)
    for t in (0, 1):
        assert list(pq[t]) == [int(v) for v in ours[t]]


def test_huffman_tables_are_annex_k():
    buf = io.BytesIO()
    Image.fromarray(np.zeros((8, 8, 3), np.uint8)).save(buf, "JPEG", quality=92, subsampling=0)
    pil = sorted(d for m, d in _segments(buf.getvalue()) if m == 0xC4)
    # libjpeg may pack all four tables into one DHT segment: split into (class/id, bits, vals)

    def split(segs):
        out = {}
        for d in segs:
            i = 0
            while i < len(d):
                tc = d[i]
                bits = list(d[i + 1:i + 17])
                n = sum(bits)
                out[tc] = (bits, list(d[i + 17:i + 17 + n]))
                i += 17 + n
        return out
    ours = split(d for m, d in _segments(O.jpeg_encode(np.zeros((8, 8, 3), np.uint8), 92)) if m == 0xC4)
    assert split(pil) == ours


@pytest.mark.parametrize("shape", [(1, 1, 3), (5, 7, 3), (64, 48, 3), (217, 333, 3), (40, 30, 1), (9, 17, 1)])
@pytest.mark.parametrize("q", [50, 92])
def test_round_trip_through_pil(shape, q):
    rng = np.random.default_rng(hash((shape, q)) & 0xFFFF)
    h, w, c = shape
    a = synth.synth_pixels(rng, w, h, gray=(c == 1)).reshape(h, w, c)
    d = O.jpeg_encode(a, q)
    im = Image.open(io.BytesIO(d))
    assert im.size == (w, h) and im.mode == ("L" if c == 1 else "RGB")
    b = np.asarray(im).reshape(h, w, c).astype(np.float64)
    # same quality through libjpeg's own encoder, 4:4:4
    buf = io.BytesIO()
    Image.fromarray(a[:, :, 0] if c == 1 else a).save(buf, "JPEG", quality=q, subsampling=0)
    ref = np.asarray(Image.open(io.BytesIO(buf.getvalue()))).reshape(h, w, c).astype(np.float64)
    psnr = lambda x: 10 * np.log10(255.0 ** 2 / max(((x - a) ** 2).mean(), 1e-9))
    assert psnr(b) > min(psnr(ref) - 1.0, 40.0)  # truncating f32 colour conversion costs a little at 1 px
    # our own decoder (pinned to libjpeg) reads the stream identically
    st, dec = O.jpeg_decode(d)
    assert st == 0 and np.array_equal(dec.reshape(h, w, c), np.asarray(im).reshape(h, w, c))


def test_fdct_dc_of_flat_block():
    # a flat block of value v has only a DC term: 8 * 8 * (v - 128) (output scaled by 8)
    import ctypes
    L = O._enc_lib()
    for v in (0, 77, 128, 255):
        s = np.full(64, v, np.uint8)
        c = np.zeros(64, np.int32)
        L.oe_fdct(s.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), c.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)))
        assert c[0] == 64 * (v - 128) and not c[1:].any()
