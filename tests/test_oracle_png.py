"""Pin the C PNG oracle (oracle/png_oracle.c) bit-exactly against PIL's PNG
decoder (lossless, so any conforming decoder gives the same samples), its
inflate against Python's zlib, and its RGBA compositing against the
reference's own known answers (image_processing.rs:846-888,
worker_files.rs:322-383)."""
import io
import os
import zlib

import numpy as np
import pytest
from PIL import Image

from datago_amd import synth
from oracle import oracle as O

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")


def _pil_expand(data: bytes) -> np.ndarray:
    """PIL decode converted the way png's Transformations::EXPAND would report it."""
    im = Image.open(io.BytesIO(data))
    trns = "transparency" in im.info
    if im.mode == "P":
        im = im.convert("RGBA" if trns else "RGB")
    elif im.mode in ("1", "L", "I", "I;16"):
        im = im.convert("LA" if trns else "L")
    elif im.mode == "RGB" and trns:
        im = im.convert("RGBA")
    a = np.asarray(im)
    return a[:, :, None] if a.ndim == 2 else a


CASES = [(k, w, h, kw) for k in synth.PNG_KINDS for (w, h) in [(1, 1), (3, 2), (17, 9), (64, 33), (255, 7)]
         for kw in ({}, {"level": 0}, {"strategy": zlib.Z_FIXED}, {"idat_max": 7, "level": 9}, {"filters": "4"})]


@pytest.mark.parametrize("case", CASES[::3], ids=lambda c: f"{c[0]}-{c[1]}x{c[2]}-{sorted(c[3].items())}")
def test_png_oracle_bit_exact_vs_pil(case):
    kind, w, h, kw = case
    data = synth.make_png(hash((kind, w, h, str(kw))) & 0xFFFF, w, h, kind, **kw)
    st, arr = O.png_decode(data)
    assert st == O.PO_OK
    ref = _pil_expand(data)
    assert arr.shape == ref.shape and np.array_equal(arr, ref)


ADAM7_CASES = [(k, w, h) for k in synth.PNG_KINDS for (w, h) in [(1, 1), (2, 3), (5, 9), (8, 8), (33, 17), (70, 41)]]


@pytest.mark.parametrize("case", ADAM7_CASES, ids=lambda c: f"{c[0]}-{c[1]}x{c[2]}")
def test_png_oracle_adam7_vs_pil(case):
    # Adam7 (PNG spec 8.2): tiny sizes leave passes empty (no filter bytes)
    kind, w, h = case
    data = synth.make_png(hash((kind, w, h, "a7")) & 0xFFFF, w, h, kind, interlace=True)
    st, arr = O.png_decode(data)
    assert st == O.PO_OK
    ref = _pil_expand(data)
    assert arr.shape == ref.shape and np.array_equal(arr, ref)


def test_png_oracle_pil_encoder():
    rng = np.random.default_rng(5)
    for mode, c in (("L", 1), ("LA", 2), ("RGB", 3), ("RGBA", 4)):
        a = synth.synth_pixels(rng, 97, 61, gray=(c <= 2))
        a = a.reshape(61, 97, -1)
        if c in (2, 4):
            a = np.concatenate([a, rng.integers(0, 256, (61, 97, 1), dtype=np.uint8)], axis=2)
        img = a[:, :, 0] if c == 1 else a
        for opt in ({}, {"optimize": True}, {"compress_level": 1}):
            data = synth.pil_png(img, **opt)
            st, arr = O.png_decode(data)
            assert st == 0 and np.array_equal(arr, _pil_expand(data)), (mode, opt)


def test_png_golden_fixtures():
    import json
    exp = json.load(open(os.path.join(GOLD, "png_expected.json")))
    import hashlib
    for name, e in exp.items():
        data = open(os.path.join(GOLD, "png", name + ".png"), "rb").read()
        st, arr = O.png_decode(data)
        assert st == e["status"], name
        if st == 0:
            assert list(arr.shape) == e["shape"], name
            assert hashlib.sha256(arr.tobytes()).hexdigest() == e["sha256"], name


@pytest.mark.parametrize("level", [0, 1, 6, 9])
def test_inflate_vs_zlib(level):
    rng = np.random.default_rng(level)
    for n in (0, 1, 100, 5000, 70000, 200000):
        raw = (rng.integers(0, 4, n) * rng.integers(0, 64, n)).astype(np.uint8).tobytes()
        z = zlib.compress(raw, level)
        st, out = O.zlib_inflate(z, n)
        assert st == O.PO_OK and out == raw


def test_inflate_corrupt():
    z = zlib.compress(bytes(range(256)) * 100, 6)
    assert O.zlib_inflate(z[:len(z) // 2], 25600)[0] == O.PO_CORRUPT
    assert O.zlib_inflate(b"\x78\x9c\xff\xff", 10)[0] == O.PO_CORRUPT
    assert O.zlib_inflate(b"\x00\x00", 10)[0] == O.PO_CORRUPT


def test_unsupported_and_corrupt():
    rng = np.random.default_rng(1)
    rows = rng.integers(0, 256, (5, 8 * 2), dtype=np.uint8)
    d16 = synth.encode_png(rows, 8, 5, 16, 0, 2, rng)
    assert O.png_info(d16)[0] == O.PO_UNSUPPORTED
    a = synth.synth_pixels(rng, 40, 30)
    d = synth.pil_png(a)
    assert O.png_info(synth.pil_png(a, interlace=1) if False else d)[0] == O.PO_OK
    assert O.png_decode(d[:60])[0] == O.PO_CORRUPT
    assert O.png_decode(b"\x89PNG\r\n\x1a\n")[0] == O.PO_CORRUPT


def test_blend_reference_known_answers():
    # image_processing.rs:846-888 and worker_files.rs:322-383
    rgba = np.array([[[255, 100, 50, 255], [200, 100, 50, 128], [255, 0, 0, 0]]], np.uint8)
    rgb = O.blend_over_gray(rgba)
    assert rgb[0, 0].tolist() == [255, 100, 50]
    assert abs(int(rgb[0, 1, 0]) - 164) <= 2 and abs(int(rgb[0, 1, 1]) - 114) <= 2 and abs(int(rgb[0, 1, 2]) - 89) <= 2
    assert rgb[0, 2].tolist() == [128, 128, 128]


def test_alpha_crop_and_resize_properties():
    # opaque RGBA resizes exactly like RGB (mul/div by 255 are identities)
    rng = np.random.default_rng(3)
    rgb = synth.synth_pixels(rng, 90, 70)
    rgba = np.concatenate([rgb, np.full((70, 90, 1), 255, np.uint8)], axis=2)
    a = O.crop_and_resize(rgba, 64, 48, O.MODE_FIR)
    b = O.crop_and_resize(rgb, 64, 48, O.MODE_FIR)
    assert np.array_equal(a[:, :, :3], b) and (a[:, :, 3] == 255).all()
