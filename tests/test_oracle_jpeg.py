"""Pin the C JPEG oracle against PIL/libjpeg-turbo (bit-exact) and against the
committed golden fixtures (tests/golden/make_golden.py)."""
import hashlib
import io
import json
import os

import numpy as np
import pytest
from PIL import Image

from datago_amd import synth
from oracle import oracle as O

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def _golden():
    with open(os.path.join(GOLD, "jpeg_expected.json")) as f:
        return json.load(f)


@pytest.mark.parametrize("name", sorted(_golden().keys()))
def test_oracle_matches_golden_fixture(name):
    exp = _golden()[name]
    data = open(os.path.join(GOLD, "jpeg", name + ".jpg"), "rb").read()
    st, arr = O.jpeg_decode(data)
    assert st == O.OJ_OK
    if exp["mode"] == "L":
        arr = arr[:, :, 0]
    assert list(arr.shape) == exp["shape"]
    assert _sha(arr) == exp["sha256"]


CASES = [(w, h, ss, gray, q)
         for (w, h) in [(1, 1), (2, 2), (3, 3), (4, 4), (5, 3), (8, 8), (17, 13), (64, 48), (100, 75)]
         for ss in ("4:2:0", "4:2:2", "4:4:4") for gray in (False, True) for q in (50, 95)
         if not (gray and ss != "4:2:0")]


@pytest.mark.parametrize("case", CASES)
def test_oracle_bit_exact_vs_pil(case):
    w, h, ss, gray, q = case
    data = synth.make_jpeg(hash(case) & 0xFFFF, w, h, q, ss, gray)
    st, arr = O.jpeg_decode(data)
    ref = np.asarray(Image.open(io.BytesIO(data)))
    if ref.ndim == 2:
        ref = ref[:, :, None]
    assert st == O.OJ_OK
    assert np.array_equal(arr, ref)


@pytest.mark.parametrize("rst", [1, 2, 5])
def test_oracle_restart_markers_vs_pil(rst):
    data = synth.make_jpeg(77 + rst, 333, 211, 88, "4:2:0", False, restart_marker_rows=rst)
    assert b"\xff\xdd" in data
    st, arr = O.jpeg_decode(data)
    assert st == O.OJ_OK
    assert np.array_equal(arr, np.asarray(Image.open(io.BytesIO(data))))


def test_oracle_rejects_cmyk_and_garbage():
    assert O.jpeg_decode(synth.make_cmyk_jpeg(0, 64, 64))[0] == O.OJ_UNSUPPORTED
    assert O.jpeg_decode(b"This is not a valid image file")[0] == O.OJ_CORRUPT


@pytest.mark.parametrize("i", range(24))
def test_oracle_progressive_matches_pil(i):
    # libjpeg's default progressive script (jpeg_simple_progression: DC first
    # Al=1, AC bands with successive approximation, refinements); sizes,
    # samplings, gray and restart intervals vary
    rng = np.random.default_rng(900 + i)
    w, h = int(rng.integers(1, 420)), int(rng.integers(1, 420))
    gray = i % 6 == 5
    data = synth.encode_jpeg(synth.synth_pixels(rng, w, h, gray), int(rng.integers(20, 101)),
                             ["4:2:0", "4:2:2", "4:4:4"][i % 3], restart_marker_blocks=(i % 4 == 1) * int(rng.integers(1, 9)),
                             progressive=True)
    st, arr = O.jpeg_decode(data)
    assert st == O.OJ_OK
    ref = np.asarray(Image.open(io.BytesIO(data)))
    assert np.array_equal(arr.reshape(ref.shape), ref)


def test_coefs_layout_counts():
    data = synth.make_jpeg(5, 33, 17, 90, "4:2:0")
    st, co = O.jpeg_coefs(data)
    assert st == O.OJ_OK
    # 4:2:0: MCU 16x16 -> 3 x 2 MCUs, 6 blocks each
    assert co.shape == (36, 64)
