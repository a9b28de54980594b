"""k_band_dec (dg_band.hip): IDCT + chroma upsampling + colour conversion +
the first horizontal Lanczos3 pass (fast_image_resize call 1,
image_processing.rs:288-298) in one kernel, the convolution on the i8
matrix cores.  Tolerance 0: the kernel must equal the oracle (and the split
IDCT -> planes -> band H path, option band_dec = 0) bit for bit in both
decode semantics, for every sampling the fused fill takes (gray, 4:4:4,
4:2:2, 4:2:0), Adobe RGB JPEGs, restart markers, progressive files, MCU-
padded edges, tile and strip-group boundaries, and every segment class."""
import numpy as np
import pytest

from datago_amd import synth
from oracle import buckets as B
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _lib():
    from datago_amd import _lib as L
    return L


def _ctx(size=1024, ratio=32, sem=0, band=1, strips=0):
    L = _lib()
    c = L.Context(0, crop_and_resize=True, default_image_size=size, downsampling_ratio=ratio, min_aspect_ratio=0.5,
                  max_aspect_ratio=2.0)
    c.set_option("decode_semantics", sem)
    c.set_option("band_dec", band)
    if strips:
        c.set_option("dec_strips", strips)
    return c


def _ref(data, tr, sem):
    with O.semantics(sem):
        st, dec = O.jpeg_decode(data)
    assert st == 0
    tw, th = tr.target_size(dec.shape[1], dec.shape[0])
    return O.crop_and_resize(dec, tw, th, O.MODE_FIR)


def _corpus(seed, n, lo, hi):
    out = []
    for i in range(n):
        rng = np.random.default_rng(seed * 1000 + i)
        ar = float(np.exp(rng.uniform(np.log(0.4), np.log(2.5))))
        short = int(rng.integers(lo, hi))
        w, h = (int(short * ar), short) if ar >= 1 else (short, int(short / ar))
        out.append(synth.make_jpeg(seed * 1000 + i, w, h, int(rng.integers(40, 98)),
                                   ["4:2:0", "4:2:2", "4:4:4"][i % 3], gray=i % 7 == 3,
                                   restart_marker_rows=1 if i % 5 == 2 else 0))
    return out


@pytest.fixture(scope="module")
def corpus():
    return _corpus(61, 30, 24, 900)


@pytest.mark.parametrize("sem", [0, 1])
def test_band_dec_bit_exact_vs_oracle_and_split_path(corpus, sem):
    tr = B.ARAwareTransform(1024, 32, 0.5, 2.0)
    fused, split = _ctx(sem=sem), _ctx(sem=sem, band=0)
    a, b = fused.decode_batch(corpus), split.decode_batch(corpus)
    assert fused.stat("band_dec_images") > len(corpus) // 2  # the fused kernel took most of them
    assert split.stat("band_dec_images") == 0
    for i, (d, (st, arr, _), (st2, arr2, _)) in enumerate(zip(corpus, a, b)):
        assert st == 0 and st2 == 0, i
        ref = _ref(d, tr, O.SEM_ZUNE if sem else O.SEM_LIBJPEG)
        assert np.array_equal(arr, ref), (i, O.jpeg_info(d))
        assert np.array_equal(arr, arr2), i


@pytest.mark.parametrize("strips", [1, 3, 64])
def test_band_dec_strip_groups(strips):
    """Strip groups restart the chroma ring (context rows recomputed at each
    group's first strip): every grouping gives the same pixels."""
    tr = B.ARAwareTransform(512, 16, 0.5, 2.0)
    datas = [synth.make_jpeg(6200 + i, w, h, 85, ss) for i, (w, h, ss) in enumerate(
        [(700, 530, "4:2:0"), (333, 801, "4:2:0"), (1201, 97, "4:2:2"), (517, 519, "4:4:4"), (64, 1000, "4:2:0")])]
    ctx = _ctx(512, 16, strips=strips)
    for d, (st, arr, _) in zip(datas, ctx.decode_batch(datas)):
        assert st == 0
        assert np.array_equal(arr, _ref(d, tr, O.SEM_LIBJPEG))


def test_band_dec_segment_classes_and_scales():
    """Upscales (7-tap windows), mild and strong downscales (both LDS segment
    classes, one and two MFMA K steps), x.5 crops after the pass, tiny and
    extreme aspect ratios."""
    tr = B.ARAwareTransform(1024, 32, 0.5, 2.0)
    sizes = [(300, 200), (520, 400), (1100, 830), (2100, 1500), (3300, 2400), (4400, 2000), (2000, 4400),
             (4100, 4100), (33, 17), (17, 33), (1300, 16), (16, 1300), (2047, 1023)]
    datas = [synth.make_jpeg(6300 + i, w, h, 70 + i, ["4:2:0", "4:2:2", "4:4:4"][i % 3], gray=i % 6 == 5)
             for i, (w, h) in enumerate(sizes)]
    ctx = _ctx()
    res = ctx.decode_batch(datas)
    assert ctx.stat("band_dec_images") >= len(datas) - 3
    for i, (d, (st, arr, _)) in enumerate(zip(datas, res)):
        assert st == 0, i
        assert np.array_equal(arr, _ref(d, tr, O.SEM_LIBJPEG)), (i, sizes[i])


def _rgb_jpeg(arr):
    """An Adobe-marker RGB JPEG (transform 0: no YCbCr conversion)."""
    import io
    from PIL import Image
    buf = io.BytesIO()
    Image.fromarray(arr).save(buf, format="JPEG", quality=90, keep_rgb=True, subsampling=0)
    return buf.getvalue()


def test_band_dec_progressive_and_rgb_colorspace():
    tr = B.ARAwareTransform(512, 16, 0.5, 2.0)
    rng = np.random.default_rng(6400)
    datas = [synth.make_jpeg(6401, 900, 600, 88, "4:2:0", progressive=True),
             synth.make_jpeg(6402, 611, 977, 75, "4:4:4", progressive=True),
             _rgb_jpeg(synth.synth_pixels(rng, 640, 420))]
    ctx = _ctx(512, 16)
    ctx.set_option("progressive", 1)
    for d, (st, arr, _) in zip(datas, ctx.decode_batch(datas)):
        assert st == 0
        assert np.array_equal(arr, _ref(d, tr, O.SEM_LIBJPEG))


def test_band_dec_full_size_properties():
    """configs[1]-size images (the oracle's decode is the slow part): the fused
    path equals the split path bit for bit and the output is the bucket."""
    datas = _corpus(62, 6, 1200, 2049)
    a, b = _ctx().decode_batch(datas), _ctx(band=0).decode_batch(datas)
    tr = B.ARAwareTransform(1024, 32, 0.5, 2.0)
    for d, (st, arr, m), (st2, arr2, _) in zip(datas, a, b):
        assert st == 0 and st2 == 0
        w, h = O.jpeg_info(d)[1:3]
        assert (m.width, m.height) == tr.target_size(w, h)
        assert np.array_equal(arr, arr2)
