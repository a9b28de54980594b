"""IDCT inputs outside what valid 8-bit JPEGs produce, bit-exact against the
oracle's 32-bit arithmetic in both decode semantics: dequantised values
beyond the signed 24-bit range (where a 24-bit-multiply IDCT would give other
pixels -- round 6 tried one) in some waves of an image and
not others, and a 16-bit quantisation table (DQT Pq = 1, SOF1).  Valid
JPEGs never get there, so the streams are built by hand: baseline Huffman
coding of chosen quantised blocks, with the standard tables taken from a
PIL-written file's DHT segments.
"""
import io
import struct

import numpy as np
import pytest
from PIL import Image

from oracle import oracle as O

pytestmark = pytest.mark.gpu

ZZ = [0, 1, 8, 16, 9, 2, 3, 10, 17, 24, 32, 25, 18, 11, 4, 5, 12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6, 7, 14,
      21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60,
      61, 54, 47, 55, 62, 63]  # zigzag index -> natural index


def _std_tables():
    """(bits, vals) of the luminance DC (class 0) and AC (class 1) tables PIL writes."""
    b = io.BytesIO()
    Image.fromarray(np.zeros((8, 8), np.uint8)).save(b, "JPEG", quality=90)
    d = b.getvalue()
    tabs, i = {}, 2
    while i < len(d) and d[i] == 0xFF and d[i + 1] != 0xDA:
        m, n = d[i + 1], struct.unpack(">H", d[i + 2:i + 4])[0]
        if m == 0xC4:
            s = d[i + 4:i + 2 + n]
            o = 0
            while o < len(s):
                tc_th = s[o]
                bits = list(s[o + 1:o + 17])
                vals = list(s[o + 17:o + 17 + sum(bits)])
                tabs[tc_th] = (bits, vals)
                o += 17 + sum(bits)
        i += 2 + n
    return tabs[0x00], tabs[0x10]


def _codes(bits, vals):
    code, k, out = 0, 0, {}
    for ln in range(1, 17):
        for _ in range(bits[ln - 1]):
            out[vals[k]] = (code, ln)
            code += 1
            k += 1
        code <<= 1
    return out


class _Bits:
    def __init__(self):
        self.acc, self.n, self.out = 0, 0, bytearray()

    def put(self, v, n):
        for i in range(n - 1, -1, -1):
            self.acc = (self.acc << 1) | ((v >> i) & 1)
            self.n += 1
            if self.n == 8:
                self.out.append(self.acc)
                if self.acc == 0xFF:
                    self.out.append(0)
                self.acc, self.n = 0, 0

    def flush(self):
        if self.n:
            self.put((1 << (8 - self.n)) - 1, 8 - self.n)
        return bytes(self.out)


def _mag(v):
    s = abs(v).bit_length()
    return s, (v if v >= 0 else v + (1 << s) - 1)


def gray_jpeg(blocks, bw, bh, q, pq16=False):
    """Baseline (or extended, 16-bit table) 1-component JPEG of bw x bh blocks
    given as quantised coefficients in natural order (int array [n, 64])."""
    (dcb, dcv), (acb, acv) = _std_tables()
    dc, ac = _codes(dcb, dcv), _codes(acb, acv)
    bw_ = _Bits()
    pred = 0
    for blk in blocks:
        z = [int(blk[ZZ[k]]) for k in range(64)]
        s, m = _mag(z[0] - pred)
        pred = z[0]
        bw_.put(*dc[s])
        bw_.put(m, s)
        run = 0
        last = max([k for k in range(1, 64) if z[k]] or [0])
        for k in range(1, last + 1):
            if z[k] == 0:
                run += 1
                continue
            while run > 15:
                bw_.put(*ac[0xF0])
                run -= 16
            s, m = _mag(z[k])
            bw_.put(*ac[(run << 4) | s])
            bw_.put(m, s)
            run = 0
        if last < 63:
            bw_.put(*ac[0x00])
    scan = bw_.flush()

    def seg(m, body):
        return bytes([0xFF, m]) + struct.pack(">H", len(body) + 2) + body

    qv = [int(q[ZZ[k]]) for k in range(64)]
    dqt = bytes([0x10 if pq16 else 0x00]) + (struct.pack(">64H", *qv) if pq16 else bytes(qv))
    sof = struct.pack(">BHHB", 8, bh * 8, bw * 8, 1) + bytes([1, 0x11, 0])
    dht = bytes([0x00]) + bytes(dcb) + bytes(dcv) + bytes([0x10]) + bytes(acb) + bytes(acv)
    sos = bytes([1, 1, 0x00, 0, 63, 0])
    return (b"\xff\xd8" + seg(0xDB, dqt) + seg(0xC1 if pq16 else 0xC0, sof) + seg(0xC4, dht) + seg(0xDA, sos) + scan
            + b"\xff\xd9")


def _blocks(rng, n, big_ranges, dc_big):
    """n blocks of small random coefficients; blocks in big_ranges ((lo, hi)
    index ranges, alternately positive and negative) get a DC of +-dc_big
    (reached by steps of at most 2047, the DC category limit) and an AC
    coefficient of magnitude up to 1023."""
    b = np.zeros((n, 64), np.int64)
    b[:, 0] = rng.integers(-60, 60, n)
    for k in range(1, 12):
        b[:, ZZ[k]] = rng.integers(-12, 13, n)
    for r, (lo, hi) in enumerate(big_ranges):
        sign = 1 if r % 2 == 0 else -1
        for i in range(lo, hi):
            b[i, 0] = sign * dc_big
            b[i, ZZ[int(rng.integers(1, 20))]] = int(rng.integers(-1023, 1024))
    # ramps: consecutive DC values may differ by at most 2047
    out = b.copy()
    for i in range(1, n):
        d = out[i, 0] - out[i - 1, 0]
        if abs(d) > 2047:
            out[i, 0] = out[i - 1, 0] + np.sign(d) * 2047
    return out


def _decode_both(blocks, bw, bh, q, pq16, sem):
    from datago_amd import _lib as L
    data = gray_jpeg(blocks, bw, bh, q, pq16)
    with O.semantics(sem):
        st, ref = O.jpeg_decode(data)
    assert st == 0
    ctx = L.Context(0, decode_semantics=sem)
    try:
        (gst, arr, _), = ctx.decode_batch([data])
    finally:
        ctx.close()
    assert gst == 0
    return arr.reshape(ref.shape), ref


@pytest.mark.parametrize("sem", [0, 1], ids=["libjpeg", "zune"])
def test_large_dequantised_inputs_exact(sem):
    """DC values of +-20000 at q = 255 (dequantised 5.1e6, beyond the 24-bit
    operand range) in two runs of blocks, one spanning two waves' boundary,
    among ordinary blocks."""
    rng = np.random.default_rng(7)
    bw, bh = 40, 48  # 1920 blocks: 30 waves of 64
    q = np.full(64, 255)
    blocks = _blocks(rng, bw * bh, [(150, 180), (1000, 1100)], 20000)
    arr, ref = _decode_both(blocks, bw, bh, q, False, sem)
    assert np.array_equal(arr, ref)


@pytest.mark.parametrize("sem", [0, 1], ids=["libjpeg", "zune"])
def test_moderately_large_coefficients_exact(sem):
    """|DC| of 9000 (past any valid 8-bit coefficient) at small q among
    ordinary blocks: the same pixels as the oracle."""
    rng = np.random.default_rng(8)
    bw, bh = 24, 24
    q = rng.integers(1, 6, 64)
    blocks = _blocks(rng, bw * bh, [(64, 70), (300, 400)], 9000)
    arr, ref = _decode_both(blocks, bw, bh, q, False, sem)
    assert np.array_equal(arr, ref)


@pytest.mark.parametrize("sem", [0, 1], ids=["libjpeg", "zune"])
def test_sixteen_bit_table(sem):
    """A 16-bit quantisation table (extended sequential, values up to 1200)."""
    rng = np.random.default_rng(9)
    bw, bh = 16, 12
    q = rng.integers(200, 1200, 64)
    blocks = _blocks(rng, bw * bh, [], 0)
    arr, ref = _decode_both(blocks, bw, bh, q, True, sem)
    assert np.array_equal(arr, ref)
