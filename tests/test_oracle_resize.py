"""Pin the resize oracle: MODE_PILLOW bit-exact vs PIL's Image.resize(LANCZOS,
box=...) two-step crop_and_resize (image_processing.rs:254-337 structure);
MODE_FIR (fast_image_resize i16 quantisation, what the GPU computes) within
3 LSB of Pillow's 22-bit quantisation."""
import hashlib
import io
import json
import os

import numpy as np
import pytest
from PIL import Image

from datago_amd import synth
from oracle import buckets as B
from oracle import oracle as O

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")
FIR_VS_PILLOW_TOL = 3  # measured max over the sample below; mean << 1


def _pil_crop_and_resize(src, tw, th):
    im = Image.fromarray(src if src.shape[2] == 3 else src[:, :, 0])
    h, w = src.shape[:2]
    if (w, h) == (tw, th):
        out = np.asarray(im)
    else:
        nw, nh = B.scaled_size(w, h, tw, th)
        l, t, cw, ch = B.fit_crop_box(nw, nh, tw, th)
        out = np.asarray(im.resize((nw, nh), Image.LANCZOS)
                         .resize((tw, th), Image.LANCZOS, box=(l, t, l + cw, t + ch)))
    return out.reshape(th, tw, -1)


@pytest.mark.parametrize("seed", range(24))
def test_pillow_mode_bit_exact(seed):
    rng = np.random.default_rng(500 + seed)
    w, h = int(rng.integers(8, 700)), int(rng.integers(8, 700))
    gray = seed % 5 == 0
    src = synth.synth_pixels(rng, w, h, gray).reshape(h, w, -1)
    t = B.ARAwareTransform(*( (1024, 32, 0.5, 2.0) if seed % 2 else (512, 32, 0.5, 2.0)))
    tw, th = t.target_size(w, h)
    ref = _pil_crop_and_resize(src, tw, th)
    out = O.crop_and_resize(src, tw, th, O.MODE_PILLOW)
    assert np.array_equal(out, ref)
    fir = O.crop_and_resize(src, tw, th, O.MODE_FIR)
    d = np.abs(fir.astype(int) - ref.astype(int))
    assert d.max() <= FIR_VS_PILLOW_TOL and d.mean() < 0.5


def test_golden_resize_fixtures_pillow_mode():
    with open(os.path.join(GOLD, "resize_expected.json")) as f:
        exp = json.load(f)
    for name, e in exp.items():
        data = open(os.path.join(GOLD, "jpeg", name + ".jpg"), "rb").read()
        st, arr = O.jpeg_decode(data)
        tw, th = e["bucket"]
        out = O.crop_and_resize(arr, tw, th, O.MODE_PILLOW)
        if arr.shape[2] == 1:
            out = out[:, :, 0]
        assert hashlib.sha256(out.tobytes()).hexdigest() == e["sha256"], name


def test_fractional_crop_is_a_resample_not_a_copy():
    # 640x480 at 512/32 -> 597x448 -> crop left = 10.5
    assert B.scaled_size(640, 480, 576, 448) == (597, 448)
    l, t, cw, ch = B.fit_crop_box(597, 448, 576, 448)
    assert l == 10.5 and t == 0.0
    rng = np.random.default_rng(3)
    src = synth.synth_pixels(rng, 597, 448)
    out = O.resample(src, 576, 448, (l, t, l + cw, t + ch))
    assert not np.array_equal(out, src[:, 10:586]) and not np.array_equal(out, src[:, 11:587])


def test_integral_crop_is_a_copy():
    rng = np.random.default_rng(4)
    src = synth.synth_pixels(rng, 592, 444)
    l, t, cw, ch = B.fit_crop_box(592, 444, 592, 432)
    # f64 crop box is not exactly integral (6.000000000000028, 431.99999999999994)
    # but the i16 coefficients quantise it to the identity: a copy
    assert l == 0.0 and abs(t - 6.0) < 1e-9 and abs(ch - 432) < 1e-9
    out = O.resample(src, 592, 432, (l, t, l + cw, t + ch))
    assert np.array_equal(out, src[6:438])


def test_portable_sin_within_one_ulp_of_libm():
    import ctypes
    import math
    L = O.lib()
    L.or_sin.restype = ctypes.c_double
    L.or_sin.argtypes = [ctypes.c_double]
    xs = np.random.default_rng(1).uniform(-30, 30, 20000)
    for x in xs:
        a, b = L.or_sin(float(x)), math.sin(float(x))
        assert abs(int(np.float64(a).view(np.int64)) - int(np.float64(b).view(np.int64))) <= 1
