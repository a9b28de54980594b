"""GPU parity: the HIP path (through the C ABI) vs the oracle, bit-exact.

Decode: both decode semantics (context option / dg_image_config
`decode_semantics`): 0 = libjpeg-turbo (oracle pinned against PIL) and 1 =
zune-jpeg 0.5.12, the reference's own decoder and the mode INTEGRATION.md
sets for the Rust drop-in (oracle SEM_ZUNE restatement, parity unpinned
against the crate itself: DESIGN.md §4).  Tests parametrised with `sem` run
in both.  Resize: the oracle's MODE_FIR restatement of fast_image_resize
(tolerance 0: the kernels use the same f64 coefficient math and i16
quantisation).  Sizes are small enough for the scalar oracle to finish in
seconds.
"""
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

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")


def _lib():
    from datago_amd import _lib as L
    return L


SEMS = [0, 1]  # decode_semantics: libjpeg-turbo, zune-jpeg (the drop-in's mode)
SEM_IDS = ["libjpeg", "zune"]


@pytest.fixture(scope="module")
def ctxs():
    """Contexts by (bucket size or 0 for decode-only, decode semantics), made once per module."""
    cache = {}

    def get(size, sem):
        if (size, sem) not in cache:
            kw = dict(crop_and_resize=True, default_image_size=size, downsampling_ratio=16 if size == 512 else 32,
                      min_aspect_ratio=0.5, max_aspect_ratio=2.0) if size else {}
            cache[(size, sem)] = _lib().Context(0, decode_semantics=sem, **kw)
        return cache[(size, sem)]
    return get


@pytest.fixture(scope="module")
def ctx_dec():
    return _lib().Context(0)


@pytest.fixture(scope="module")
def ctx512():
    return _lib().Context(0, crop_and_resize=True, default_image_size=512, downsampling_ratio=16,
                          min_aspect_ratio=0.5, max_aspect_ratio=2.0)


@pytest.fixture(scope="module")
def ctx1024():
    return _lib().Context(0, crop_and_resize=True, default_image_size=1024, downsampling_ratio=32,
                          min_aspect_ratio=0.5, max_aspect_ratio=2.0)


def _golden_files():
    with open(os.path.join(GOLD, "jpeg_expected.json")) as f:
        names = sorted(json.load(f).keys())
    return [(n, open(os.path.join(GOLD, "jpeg", n + ".jpg"), "rb").read()) for n in names]


def _oracle_decoded(data, sem=0):
    with O.semantics(sem):
        st, dec = O.jpeg_decode(data)
    assert st == 0
    return dec


def _oracle_resized(data, tw, th, sem=0):
    return O.crop_and_resize(_oracle_decoded(data, sem), tw, th, O.MODE_FIR)


def _rand_jpegs(seed, n, maxdim=700, rst=False):
    out = []
    for i in range(n):
        rng = np.random.default_rng(seed * 1000 + i)
        w, h = int(rng.integers(1, maxdim)), int(rng.integers(1, maxdim))
        ss = ["4:2:0", "4:2:2", "4:4:4"][i % 3]
        r = ([0, 1, 2][i % 3] if rst else 0)
        out.append(synth.encode_jpeg(synth.synth_pixels(rng, w, h, i % 9 == 4), int(rng.integers(40, 101)), ss,
                                     restart_marker_rows=r))
    return out


def test_decode_only_golden_bit_exact(ctx_dec):
    files = _golden_files()
    res = ctx_dec.decode_batch([d for _, d in files])
    exp = json.load(open(os.path.join(GOLD, "jpeg_expected.json")))
    for (name, data), (st, arr, meta) in zip(files, res):
        assert st == 0, (name, st)
        a = arr[:, :, 0] if exp[name]["mode"] == "L" else arr
        assert list(a.shape) == exp[name]["shape"], name
        assert hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest() == exp[name]["sha256"], name
    assert ctx_dec.stat("write_mismatch") == 0


@pytest.mark.parametrize("sem", SEMS, ids=SEM_IDS)
def test_decode_only_random_bit_exact_vs_oracle(ctxs, sem):
    datas = _rand_jpegs(1, 24, rst=True)
    res = ctxs(0, sem).decode_batch(datas)
    for i, (d, (st, arr, meta)) in enumerate(zip(datas, res)):
        ref = _oracle_decoded(d, sem)
        assert st == 0
        assert arr.shape == ref.shape, i
        assert np.array_equal(arr, ref), (i, int((arr != ref).sum()))
        assert (meta.original_width, meta.original_height) == (ref.shape[1], ref.shape[0])


def test_crop_resize_golden_bit_exact(ctx512):
    files = _golden_files()
    res = ctx512.decode_batch([d for _, d in files])
    t = B.ARAwareTransform(512, 16, 0.5, 2.0)
    for (name, data), (st, arr, meta) in zip(files, res):
        assert st == 0, name
        w, h = O.jpeg_info(data)[1:3]
        tw, th = t.target_size(w, h)
        assert (meta.width, meta.height) == (tw, th)
        ref = _oracle_resized(data, tw, th)
        assert arr.shape == ref.shape, name
        d = np.abs(arr.astype(int) - ref.astype(int))
        assert d.max() == 0, (name, int(d.max()), int((d > 0).sum()))


@pytest.mark.parametrize("sem", SEMS, ids=SEM_IDS)
def test_crop_resize_random_1024(ctxs, sem):
    ctx = ctxs(1024, sem)
    datas = _rand_jpegs(2, 16, maxdim=1400)
    res = ctx.decode_batch(datas)
    t = B.ARAwareTransform(1024, 32, 0.5, 2.0)
    for i, (data, (st, arr, meta)) in enumerate(zip(datas, res)):
        assert st == 0
        w, h = O.jpeg_info(data)[1:3]
        tw, th = t.target_size(w, h)
        ref = _oracle_resized(data, tw, th, sem)
        assert arr.shape == ref.shape
        assert np.array_equal(arr, ref), (i, (w, h), (tw, th))
    assert ctx.stat("write_mismatch") == 0


def test_fractional_crop_case(ctx512):
    # 640x480 into 512/32 buckets: 597x448 then crop left 10.5
    L = _lib()
    ctx = L.Context(0, crop_and_resize=True, default_image_size=512, downsampling_ratio=32,
                    min_aspect_ratio=0.5, max_aspect_ratio=2.0)
    data = synth.make_jpeg(9, 640, 480, 90)
    st, arr, meta = ctx.decode_one(data)
    assert st == 0 and (meta.width, meta.height) == (576, 448)
    assert np.array_equal(arr, _oracle_resized(data, 576, 448))


def test_subsequence_sizes_agree(ctx_dec):
    datas = _rand_jpegs(3, 6, maxdim=900)
    L = _lib()
    base = [a for _, a, _ in ctx_dec.decode_batch(datas)]
    for sb in (128, 512, 4096, 16384):
        ctx = L.Context(0)
        ctx.set_option("sub_bits", sb)
        for (st, a, _), b in zip(ctx.decode_batch(datas), base):
            assert st == 0 and np.array_equal(a, b), sb
        assert ctx.stat("write_mismatch") == 0


@pytest.mark.parametrize("bands,slots,sem", [(1, 1, 0), (3, 2, 1), (8, 3, 0), (64, 4, 1)])
def test_band_and_slot_options_bit_exact(bands, slots, sem):
    # the band H kernel's rows per workgroup (hb_bands) and the batches in
    # flight (slots) change only the partitioning: outputs stay bit-exact
    L = _lib()
    ctx = L.Context(0, crop_and_resize=True, default_image_size=1024, downsampling_ratio=32,
                    min_aspect_ratio=0.5, max_aspect_ratio=2.0, decode_semantics=sem)
    ctx.set_option("hb_bands", bands)
    ctx.set_option("slots", slots)
    datas = _rand_jpegs(5, 6, maxdim=1300)
    t = B.ARAwareTransform(1024, 32, 0.5, 2.0)
    for _ in range(2):  # consecutive batches cycle through the slots
        for data, (st, arr, meta) in zip(datas, ctx.decode_batch(datas)):
            assert st == 0
            w, h = O.jpeg_info(data)[1:3]
            assert np.array_equal(arr, _oracle_resized(data, *t.target_size(w, h), sem)), (bands, slots, (w, h))


@pytest.mark.parametrize("sub_bits", [0, 512, 2048, 8192])
def test_entropy_decode_once_matches(sub_bits):
    """Option entropy_once: k_huff_sync stages every coefficient and
    k_huff_scatter writes the blocks (no second decode).  Outputs must equal
    the default two-pass path and the oracle bit for bit, with restart
    markers (owned / unowned at range ends), gray, 4:2:2 and 4:4:4."""
    L = _lib()
    datas = _rand_jpegs(8, 10, maxdim=1200) + _rand_jpegs(9, 8, maxdim=900, rst=True)
    datas.append(synth.make_jpeg(88, 2000, 1500, 95, "4:2:0", False, restart_marker_rows=1))
    ctx = L.Context(0)
    ctx.set_option("entropy_once", 1)
    if sub_bits:
        ctx.set_option("sub_bits", sub_bits)
    for i, (d, (st, arr, _)) in enumerate(zip(datas, ctx.decode_batch(datas))):
        assert st == 0, i
        ost, ref = O.jpeg_decode(d)
        assert np.array_equal(arr.reshape(ref.shape), ref), (i, sub_bits)


@pytest.mark.parametrize("meta_pull,plan_threads", [(0, 1), (1, 1), (2, 4), (0, 7)])
def test_upload_and_planning_options_bit_exact(meta_pull, plan_threads):
    """The descriptor/input upload (meta_pull: GPU-pulled from page-locked
    staging, or hipMemcpyAsync) and the planning workers (plan_threads) move
    no pixel: host-in batches (inputs pulled too) and device-resident batches
    both equal the oracle."""
    L = _lib()
    ctx = L.Context(0, crop_and_resize=True, default_image_size=512, downsampling_ratio=16,
                    min_aspect_ratio=0.5, max_aspect_ratio=2.0, decode_semantics=1)
    ctx.set_option("meta_pull", meta_pull)
    ctx.set_option("plan_threads", plan_threads)
    datas = _rand_jpegs(41, 80, maxdim=500)  # > 2 x 32 images: the workers take part
    t = B.ARAwareTransform(512, 16, 0.5, 2.0)
    refs = [_oracle_resized(d, *t.target_size(*O.jpeg_info(d)[1:3]), 1) for d in datas]
    for _ in range(2):
        for ref, (st, arr, meta) in zip(refs, ctx.decode_batch(datas)):
            assert st == 0
            assert np.array_equal(arr, ref), (meta_pull, plan_threads)
    assert ctx.stat("meta_bytes") > 0


@pytest.mark.parametrize("sub_bits,split", [(1024, 1), (4096, 1), (8192, 1), (8192, 0)])
def test_write_split_bit_exact(sub_bits, split):
    """Option write_split: k_huff_write decodes each range as two halves, the
    second from the sync pass's half-way checkpoint with the blocks and DC
    sums before it taken from the checkpoint's tail.  Bit-exact against the
    oracle, with restart markers (no split), gray, 4:2:2 and 4:4:4, ranges
    shorter than half a subsequence, and no write mismatch."""
    L = _lib()
    datas = _rand_jpegs(12, 12, maxdim=1400) + _rand_jpegs(13, 4, maxdim=900, rst=True)
    datas.append(synth.make_jpeg(89, 2400, 1600, 92, "4:2:0", False))
    datas.append(synth.make_jpeg(90, 1800, 1200, 60, "4:4:4", False))
    ctx = L.Context(0)
    ctx.set_option("write_split", split)
    ctx.set_option("sub_bits", sub_bits)
    for i, (d, (st, arr, _)) in enumerate(zip(datas, ctx.decode_batch(datas))):
        assert st == 0, i
        ost, ref = O.jpeg_decode(d)
        assert np.array_equal(arr.reshape(ref.shape), ref), (i, sub_bits)
    assert ctx.stat("write_mismatch") == 0


def test_band_and_slot_options_validated():
    L = _lib()
    ctx = L.Context(0)
    for k, v in (("hb_bands", 0), ("hb_bands", 65), ("slots", 0), ("slots", 7), ("inf_decode", -1),
                 ("inf_decode", 10), ("inf_decode", 29), ("uf_units", 0), ("uf_units", 3), ("plan_threads", 0), ("inf_chunk", 1000),
                 ("inf_chunk", 2048), ("inf_stage3", 12), ("sub_auto", 3000), ("meta_pull", 3)):
        with pytest.raises(Exception):
            ctx.set_option(k, v)


def test_forced_bucket_alignment(ctx512):
    # worker_wds.rs:68-76: later members are forced into the first image's bucket
    t = ctx512.buckets
    k = t.find_key("1.000")
    data = synth.make_jpeg(11, 300, 200, 90)
    st, arr, meta = ctx512.decode_one(data, forced_bucket=k)
    assert st == 0 and (meta.width, meta.height) == (512, 512) and meta.bucket == k
    assert np.array_equal(arr, _oracle_resized(data, 512, 512))


def test_exact_size_is_a_copy(ctx512):
    data = synth.make_jpeg(12, 512, 512, 90)
    st, arr, meta = ctx512.decode_one(data)
    assert st == 0
    assert np.array_equal(arr, O.jpeg_decode(data)[1])


def test_status_codes(ctx512):
    import io as _io
    L = _lib()
    good = synth.make_jpeg(13, 64, 64, 90)
    cmyk = synth.make_cmyk_jpeg(0, 64, 64)  # valid, outside the GPU path
    png = _io.BytesIO()  # 16-bit PNG: valid, outside the GPU path (the Rust glue keeps its CPU decode)
    Image.fromarray(np.arange(64, dtype=np.uint16).reshape(8, 8) * 1000).save(png, format="PNG")
    trunc = synth.make_jpeg(14, 300, 300, 90)[:1500]
    res = ctx512.decode_batch([good, b"This is not a valid image file", cmyk, png.getvalue(), trunc, good])
    sts = [r[0] for r in res]
    assert sts == [L.DG_OK, L.DG_ERR_CORRUPT, L.DG_ERR_UNSUPPORTED, L.DG_ERR_UNSUPPORTED, L.DG_ERR_CORRUPT, L.DG_OK]
    assert np.array_equal(res[0][1], res[5][1])


def test_tiny_and_extreme_images():
    # test_datago_edge_cases.py:100-172 (1x1, 1000x10, 10x1000 at 224/16 buckets)
    L = _lib()
    ctx = L.Context(0, crop_and_resize=True, default_image_size=224, downsampling_ratio=16,
                    min_aspect_ratio=0.5, max_aspect_ratio=2.0)
    datas = [synth.make_jpeg(20, 1, 1, 90), synth.make_jpeg(21, 1000, 10, 90), synth.make_jpeg(22, 10, 1000, 90)]
    t = B.ARAwareTransform(224, 16, 0.5, 2.0)
    for data, (st, arr, meta) in zip(datas, ctx.decode_batch(datas)):
        assert st == 0
        w, h = O.jpeg_info(data)[1:3]
        tw, th = t.target_size(w, h)
        assert 0.5 <= meta.width / meta.height <= 2.0
        assert np.array_equal(arr, _oracle_resized(data, tw, th))


def test_gray_to_rgb8():
    L = _lib()
    ctx = L.Context(0, crop_and_resize=True, default_image_size=256, downsampling_ratio=16,
                    min_aspect_ratio=0.5, max_aspect_ratio=2.0, image_to_rgb8=True)
    data = synth.make_jpeg(23, 333, 250, 90, gray=True)
    st, arr, meta = ctx.decode_one(data)
    assert st == 0 and meta.channels == 3 and arr.shape[2] == 3
    t = B.ARAwareTransform(256, 16, 0.5, 2.0)
    tw, th = t.target_size(333, 250)
    ref = _oracle_resized(data, tw, th)
    assert np.array_equal(arr, np.repeat(ref, 3, axis=2))


def test_large_full_size_properties(ctx1024):
    # BASELINE configs[1] sizes (short side up to 2048): size-independent checks
    datas = [synth.make_jpeg(30 + i, w, h, 85, ss) for i, (w, h, ss) in
             enumerate([(2048, 1536, "4:2:0"), (1600, 2600, "4:2:2"), (2300, 1100, "4:4:4")])]
    res = ctx1024.decode_batch(datas)
    res2 = ctx1024.decode_batch(datas)
    t = B.ARAwareTransform(1024, 32, 0.5, 2.0)
    for data, (st, arr, meta), (st2, arr2, _) in zip(datas, res, res2):
        assert st == 0 and st2 == 0
        assert np.array_equal(arr, arr2)  # deterministic
        w, h = O.jpeg_info(data)[1:3]
        assert (meta.width, meta.height) == t.target_size(w, h)
        # the decode stage against PIL directly (libjpeg-turbo) via the oracle-equivalent resize
        pil = np.asarray(Image.open(io.BytesIO(data)))
        ref = O.crop_and_resize(pil, meta.width, meta.height, O.MODE_FIR)
        assert np.array_equal(arr, ref)


# Horizontal-pass kernel classes: register-resident weights for
# ksize <= 8 / 16 / 32, weights from global beyond that, and the direct kernel
# when the source segment of a 256-column tile exceeds LDS; colour images use
# the fused upsample + colour fill, gray the byte fill.
H_CLASS_CASES = [
    (300, 200, "4:2:0", False),   # upscale: ksize 7
    (700, 520, "4:2:2", False),   # mild downscale: <= 16
    (2000, 1500, "4:4:4", False), # ~3.4x: <= 32
    (4000, 3000, "4:2:0", False), # ~6.8x: generic weights
    (6400, 4000, "4:2:0", False), # ~10x: direct kernel
    (1999, 1001, "4:2:0", True),  # gray, odd sizes
    (7000, 900, "4:2:2", False),  # AR beyond the bucket range, very wide
]


@pytest.mark.parametrize("sem", SEMS, ids=SEM_IDS)
@pytest.mark.parametrize("case", H_CLASS_CASES, ids=lambda c: f"{c[0]}x{c[1]}_{c[2]}_{'L' if c[3] else 'RGB'}")
def test_h_pass_classes_bit_exact(ctxs, case, sem):
    w, h, ss, gray = case
    data = synth.make_jpeg(40 + w % 97, w, h, 88, ss, gray=gray)
    st, arr, meta = ctxs(512, sem).decode_one(data)
    assert st == 0
    t = B.ARAwareTransform(512, 16, 0.5, 2.0)
    tw, th = t.target_size(w, h)
    ref = _oracle_resized(data, tw, th, sem)
    assert arr.shape == ref.shape
    d = np.abs(arr.astype(int) - ref.astype(int))
    assert d.max() == 0, (int(d.max()), int((d > 0).sum()), np.argwhere(d > 0)[:4].tolist())


# Crop folding: an integral crop offset is a window of call 1's
# outputs, a fractional one keeps call 2's sub-pixel pass; without a call-1
# pass on an axis the window is a plain offset (these sizes have scale 1 on
# one or both axes at the 512/16 buckets: 592x432 / 432x592 / 512x512).
CROP_CASES = [
    (700, 432, False),   # scale 1, integral x crop: no pass at all, offset copy
    (701, 432, False),   # scale 1, x.5 crop: H2 alone
    (432, 700, True),    # gray, integral y crop
    (432, 701, False),   # y.5 crop: V2 alone
    (1184, 865, False),  # downscale, y crop window folded into V1
    (1185, 864, True),   # gray, downscale
    (640, 480, False),   # 592x444 -> crop top 6 (integral, folded into V1)
]


@pytest.mark.parametrize("sem", SEMS, ids=SEM_IDS)
@pytest.mark.parametrize("case", CROP_CASES, ids=lambda c: f"{c[0]}x{c[1]}_{'L' if c[2] else 'RGB'}")
def test_crop_folding_bit_exact(ctxs, case, sem):
    w, h, gray = case
    data = synth.make_jpeg(60 + w % 89 + h % 7, w, h, 90, "4:2:0", gray=gray)
    st, arr, meta = ctxs(512, sem).decode_one(data)
    assert st == 0
    t = B.ARAwareTransform(512, 16, 0.5, 2.0)
    tw, th = t.target_size(w, h)
    assert (meta.width, meta.height) == (tw, th)
    ref = _oracle_resized(data, tw, th, sem)
    assert arr.shape == ref.shape
    d = np.abs(arr.astype(int) - ref.astype(int))
    assert d.max() == 0, (int(d.max()), int((d > 0).sum()))


def test_decode_one_coalesces_concurrent_callers(ctx512):
    # concurrent single-image calls (one per tokio task in the
    # reference) are merged into shared GPU batches, results unchanged
    import threading
    L = _lib()
    ctx = L.Context(0, crop_and_resize=True, default_image_size=512, downsampling_ratio=16,
                    min_aspect_ratio=0.5, max_aspect_ratio=2.0)
    ctx.set_option("coalesce_us", 20000)
    datas = _rand_jpegs(7, 32, maxdim=500)
    res = [None] * len(datas)

    def work(k):
        for i in range(k, len(datas), 8):
            res[i] = ctx.decode_one(datas[i])

    th = [threading.Thread(target=work, args=(k,)) for k in range(8)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    t = B.ARAwareTransform(512, 16, 0.5, 2.0)
    for data, (st, arr, meta) in zip(datas, res):
        assert st == 0
        w, h = O.jpeg_info(data)[1:3]
        assert np.array_equal(arr, _oracle_resized(data, *t.target_size(w, h)))
    assert ctx.stat("coalesced_images") == len(datas)
    assert ctx.stat("coalesced_batches") < len(datas)  # merged


def _content(kind, rng, w, h, gray):
    """Entropy regimes the synthetic corpus alone does not stress (VERDICT r1
    weak item 11): flat low-detail images (short, EOB-heavy codes: the
    slowest entropy workgroups), uniform noise (long codes, many AC symbols),
    hard-edged stripes/text-like blocks, and the bench's own gradient+noise."""
    if kind == "flat":
        yy, xx = np.mgrid[0:h, 0:w]
        base = (96 + 64 * np.sin(xx / max(w, 1) * 3.1) * np.cos(yy / max(h, 1) * 2.3)).astype(np.float32)
        arr = np.repeat(base[:, :, None], 1 if gray else 3, axis=2) + (0 if gray else np.array([0, 20, -20]))
        arr = arr.clip(0, 255).astype(np.uint8)
        return arr[:, :, 0] if gray else arr
    if kind == "noise":
        return rng.integers(0, 256, (h, w) if gray else (h, w, 3), dtype=np.uint8)
    if kind == "edges":
        yy, xx = np.mgrid[0:h, 0:w]
        m = (((xx // 7) + (yy // 11)) % 2 * 255).astype(np.uint8)
        return m if gray else np.stack([m, 255 - m, (m // 2 + 64).astype(np.uint8)], axis=2)
    return synth.synth_pixels(rng, w, h, gray)


FULL_CASES = [  # (content, w, h, quality, subsampling, gray): configs[1] sizes, short side 256..2048
    ("flat", 2048, 1536, 35, "4:2:0", False), ("flat", 1024, 2300, 60, "4:2:2", False),
    ("noise", 1500, 1100, 95, "4:2:0", False), ("noise", 640, 1500, 90, "4:4:4", False),
    ("edges", 1800, 900, 80, "4:2:0", False), ("edges", 913, 1219, 75, "4:2:0", True),
    ("synth", 2600, 1100, 88, "4:2:0", False), ("synth", 1279, 1935, 92, "4:4:4", False),
    ("flat", 777, 2048, 50, "4:2:0", True), ("synth", 256, 611, 75, "4:2:2", False),
    ("noise", 2047, 257, 85, "4:2:2", False), ("edges", 1333, 1333, 95, "4:4:4", False),
]


@pytest.mark.parametrize("sem", SEMS, ids=SEM_IDS)
def test_full_size_regimes_bit_exact_vs_oracle(ctxs, sem):
    """Full configs[1]-size images end to end (decode + bucket + crop/resize at
    1024/32), every regime in one batch, bit-exact against the oracle in
    both decode semantics."""
    ctx = ctxs(1024, sem)
    datas = []
    for i, (kind, w, h, q, ss, gray) in enumerate(FULL_CASES):
        rng = np.random.default_rng(900 + i)
        datas.append(synth.encode_jpeg(_content(kind, rng, w, h, gray), q, ss))
    res = ctx.decode_batch(datas)
    t = B.ARAwareTransform(1024, 32, 0.5, 2.0)
    for k, (data, (st, arr, meta)) in enumerate(zip(datas, res)):
        assert st == 0, (k, FULL_CASES[k])
        dec = _oracle_decoded(data, sem)
        ref = O.crop_and_resize(dec, *t.target_size(dec.shape[1], dec.shape[0]), O.MODE_FIR)
        assert np.array_equal(arr, ref), FULL_CASES[k]
    assert ctx.stat("write_mismatch") == 0


def test_zune_bench_pool_sample_bit_exact(ctxs):
    """A slice of the bench's own configs[1] pool (bench.py's corpus: seeded
    mixed aspect ratios, short side 256..2048, q 75..95, 80/10/10 % 4:2:0 /
    4:2:2 / 4:4:4, 5 % gray) at 1024/32 in zune mode, the mode the headline
    is measured in: every output bit-exact against the SEM_ZUNE oracle."""
    ctx = ctxs(1024, 1)
    datas = synth.mixed_corpus(2, 4096, lo=0, hi=16)  # bench.py's configs[1] pool (seed 2, 4,096 images)
    t = B.ARAwareTransform(1024, 32, 0.5, 2.0)
    for k, (data, (st, arr, meta)) in enumerate(zip(datas, ctx.decode_batch(datas))):
        assert st == 0, k
        dec = _oracle_decoded(data, 1)
        assert np.array_equal(arr, O.crop_and_resize(dec, *t.target_size(dec.shape[1], dec.shape[0]), O.MODE_FIR)), k


@pytest.mark.parametrize("sub_bits", [512, 8192])
def test_full_size_regimes_subsequence_sizes(sub_bits):
    """The same regimes through other subsequence sizes: decode-only outputs equal the default's."""
    L = _lib()
    datas = []
    for i, (kind, w, h, q, ss, gray) in enumerate(FULL_CASES[:6]):
        rng = np.random.default_rng(900 + i)
        datas.append(synth.encode_jpeg(_content(kind, rng, w, h, gray), q, ss))
    a = L.Context(0).decode_batch(datas)
    c = L.Context(0)
    c.set_option("sub_bits", sub_bits)
    for (sa, xa, _), (sb, xb, _) in zip(a, c.decode_batch(datas)):
        assert sa == 0 and sb == 0 and np.array_equal(xa, xb)


def test_fused_idct_option_bit_exact():
    """Option idct_fused (off by default: k_huff_write 1.7 -> 12 ms measured,
    DESIGN.md §5): completed blocks IDCT-ed inside the entropy write kernel's
    cooperative flush, carried-in and few-lane blocks through k_idct_list.
    Same pixels as the separate k_idct, every subsequence size."""
    L = _lib()
    datas = _rand_jpegs(12, 9, maxdim=900) + [synth.make_jpeg(77, 3, 2, 90, "4:2:0"),
                                              synth.make_jpeg(78, 1, 1, 90, "4:4:4", gray=True)]
    base = [a for _, a, _ in L.Context(0).decode_batch(datas)]
    for sb in (0, 512, 16384):
        c = L.Context(0)
        c.set_option("idct_fused", 1)
        if sb:
            c.set_option("sub_bits", sb)
        for k, ((st, a, _), b) in enumerate(zip(c.decode_batch(datas), base)):
            assert st == 0 and np.array_equal(a, b), (sb, k)


def test_host_output_copies_threaded_equal():
    """Host-out batches copy outputs to the caller's buffers on up to
    `copy_threads` threads in 1 MiB pieces; 1 and 8 threads give identical
    bytes and both equal the oracle (large 1024-bucket outputs, so the
    threaded path really splits)."""
    from datago_amd import _lib as L
    datas = [synth.make_jpeg(700 + i, 1900 - 97 * i, 1200 + 133 * i, 90, ["4:2:0", "4:4:4", "4:2:2"][i % 3])
             for i in range(6)]
    t = B.ARAwareTransform(1024, 32, 0.5, 2.0)
    outs = {}
    for nt in (1, 8):
        ctx = L.Context(0, crop_and_resize=True, default_image_size=1024, downsampling_ratio=32,
                        min_aspect_ratio=0.5, max_aspect_ratio=2.0)
        ctx.set_option("copy_threads", nt)
        outs[nt] = ctx.decode_batch(datas)
    for d, (s1, a1, _), (s8, a8, _) in zip(datas, outs[1], outs[8]):
        assert s1 == 0 and s8 == 0 and np.array_equal(a1, a8)
        _, dec = O.jpeg_decode(d)
        assert np.array_equal(a8, O.crop_and_resize(dec, *t.target_size(dec.shape[1], dec.shape[0]), O.MODE_FIR))


def test_fused_hv_resize_equal():
    """Option hv_fused routes colour JPEGs whose first H and V passes fit
    k_resize_hv (H taps <= 15, V taps <= 24, source span <= 320 px per 128
    output columns) through the fused kernel: outputs equal the two-pass
    path and the oracle byte for byte (downscales 1.0-2.3x, tall and wide
    crops, every subsampling)."""
    from datago_amd import _lib as L
    dims = [(1100, 1500), (2048, 1536), (1536, 2048), (1300, 700), (900, 1800), (2300, 2300), (1030, 1030)]
    datas = [synth.make_jpeg(900 + i, w, h, 88, ["4:2:0", "4:4:4", "4:2:2"][i % 3]) for i, (w, h) in enumerate(dims)]
    t = B.ARAwareTransform(1024, 32, 0.5, 2.0)
    outs = {}
    for hv in (0, 1):
        ctx = L.Context(0, crop_and_resize=True, default_image_size=1024, downsampling_ratio=32,
                        min_aspect_ratio=0.5, max_aspect_ratio=2.0)
        ctx.set_option("hv_fused", hv)
        outs[hv] = ctx.decode_batch(datas)
    for d, (s0, a0, _), (s1, a1, _) in zip(datas, outs[0], outs[1]):
        assert s0 == 0 and s1 == 0 and np.array_equal(a0, a1)
        _, dec = O.jpeg_decode(d)
        assert np.array_equal(a1, O.crop_and_resize(dec, *t.target_size(dec.shape[1], dec.shape[0]), O.MODE_FIR))


@pytest.mark.parametrize("v_tile", [2, 4, 8])
def test_v_tile_bit_exact(v_tile):
    """Option v_tile: the V passes on R-row column tiles (k_resize_vt; VERDICT
    r5 item 4) equal the one-thread-per-16-bytes kernel (v_tile 0) and the
    oracle byte for byte: colour and gray JPEGs, PNG with alpha (the alpha
    programs around the convolution), x.5 crops (call 2's 6-tap V pass),
    upscales, and 16x downscales whose tile spans need several weight-table
    windows (> kVtWCap / R pairs), rows not a multiple of R, rows narrower
    than one 64-unit chunk and wider than several."""
    from datago_amd import _lib as L
    dims = [(1100, 1500), (2048, 1536), (333, 777), (1300, 700), (5, 2000), (2047, 3), (640, 480)]
    datas = [synth.make_jpeg(950 + i, w, h, 88, ["4:2:0", "4:4:4", "4:2:2", "4:2:0"][i % 4], gray=i % 4 == 3)
             for i, (w, h) in enumerate(dims)]
    datas += [synth.make_png(960, 517, 1203, "RGBA", level=1), synth.make_png(961, 900, 333, "L", level=1)]
    for size, ratio in ((1024, 32), (128, 16)):
        t = B.ARAwareTransform(size, ratio, 0.5, 2.0)
        outs = {}
        for vt in (0, v_tile):
            ctx = L.Context(0, crop_and_resize=True, default_image_size=size, downsampling_ratio=ratio,
                            min_aspect_ratio=0.5, max_aspect_ratio=2.0)
            ctx.set_option("v_tile", vt)
            outs[vt] = ctx.decode_batch(datas)
            ctx.close()
        for d, (s0, a0, _), (s1, a1, _) in zip(datas, outs[0], outs[v_tile]):
            assert s0 == 0 and s1 == 0 and a0.shape == a1.shape and np.array_equal(a0, a1), (size, a0.shape)
            if d[:4] == b"\x89PNG":
                continue  # (the PNG suites pin PNG resizes to the oracle; here: equal to v_tile 0)
            _, dec = O.jpeg_decode(d)
            assert np.array_equal(a1, O.crop_and_resize(dec, *t.target_size(dec.shape[1], dec.shape[0]), O.MODE_FIR))


@pytest.mark.parametrize("sem", SEMS, ids=SEM_IDS)
def test_h_planar_bit_exact(sem):
    """Option h_planar: the fused 8- and 16-tap band H passes over planar
    u16-pair segments (k_resize_hbp; the 4:2:0 zune fill in packed 16-bit
    arithmetic) equal k_resize_hb (h_planar 0) and the oracle byte for byte:
    every fill class (4:2:0 / 4:2:2 / 4:4:4, gray, an RGB-transform JPEG on
    the generic fill), widths whose padded chroma row ends inside the
    segment (zune's last-pair quirk) or past it, odd window starts, 1x-2.5x
    downscales (both planar classes) and wider ones (k_resize_hb's 32-tap
    class beside them), upscales, x.5 crops, with and without the next-band
    prefetch."""
    from datago_amd import _lib as L
    dims = [(1100, 1500), (2048, 1536), (333, 777), (1300, 700), (1024, 1024), (1040, 1568), (2600, 1100),
            (777, 2048), (1536, 1536), (903, 1601), (2304, 1296), (3000, 1000)]
    subs = ["4:2:0", "4:2:0", "4:2:2", "4:4:4", "4:2:0", "4:2:0", "4:2:0", "4:2:2", "4:4:4", "4:2:0", "4:2:0",
            "4:2:0"]
    datas = [synth.make_jpeg(1950 + i, w, h, 80 + i, subs[i], gray=i == 6) for i, (w, h) in enumerate(dims)]
    rgb = io.BytesIO()
    Image.fromarray(synth.synth_pixels(np.random.default_rng(3), 1200, 900, False)).save(
        rgb, "JPEG", quality=90, keep_rgb=True)
    datas.append(rgb.getvalue())
    for size, ratio in ((1024, 32), (512, 16)):
        t = B.ARAwareTransform(size, ratio, 0.5, 2.0)
        outs = {}
        for hp, pf in ((0, 1), (1, 1), (1, 0)):
            ctx = L.Context(0, crop_and_resize=True, default_image_size=size, downsampling_ratio=ratio,
                            min_aspect_ratio=0.5, max_aspect_ratio=2.0, decode_semantics=sem)
            ctx.set_option("h_planar", hp)
            ctx.set_option("h_prefetch", pf)
            outs[(hp, pf)] = ctx.decode_batch(datas)
            ctx.close()
        for k, d in enumerate(datas):
            s0, a0, _ = outs[(0, 1)][k]
            assert s0 == 0
            for key in ((1, 1), (1, 0)):
                s1, a1, _ = outs[key][k]
                assert s1 == 0 and a1.shape == a0.shape and np.array_equal(a0, a1), (size, k, key)
            dec = _oracle_decoded(d, sem)
            assert np.array_equal(a0, O.crop_and_resize(dec, *t.target_size(dec.shape[1], dec.shape[0]),
                                                        O.MODE_FIR)), (size, k)


@pytest.mark.parametrize("sub_bits,lead", [(0, -1), (1024, -1), (4096, 0), (8192, -1), (2048, 6144)])
def test_sync2_bit_exact(sub_bits, lead):
    """Option sync2: k_huff_sync2 runs two lead-in + range chains per lane
    (SyncChain, dg_entropy.h; tests/native/emu.cpp checks each pair against
    lead_in + decode_range).  Bit-exact against the oracle and against the
    one-chain kernel -- with restart markers, gray, 4:2:2 / 4:4:4, images of
    fewer subsequences than a workgroup and of many workgroups -- with no
    write mismatch."""
    L = _lib()
    datas = _rand_jpegs(14, 12, maxdim=1400) + _rand_jpegs(15, 4, maxdim=900, rst=True)
    datas.append(synth.make_jpeg(91, 2400, 1600, 92, "4:2:0", False))
    datas.append(synth.make_jpeg(92, 1800, 1200, 60, "4:4:4", False))
    datas.append(synth.make_jpeg(93, 3000, 2000, 95, "4:2:0", False, restart_marker_rows=2))
    outs = {}
    for two in (0, 1):
        ctx = L.Context(0)
        ctx.set_option("sync2", two)
        if sub_bits:
            ctx.set_option("sub_bits", sub_bits)
        if lead >= 0:
            ctx.set_option("lead_bits", lead)
        outs[two] = ctx.decode_batch(datas)
        assert ctx.stat("write_mismatch") == 0
        ctx.close()
    for i, (d, (s0, a0, _), (s1, a1, _)) in enumerate(zip(datas, outs[0], outs[1])):
        assert s0 == 0 and s1 == 0, i
        assert np.array_equal(a0, a1), (i, sub_bits)
        ost, ref = O.jpeg_decode(d)
        assert np.array_equal(a1.reshape(ref.shape), ref), (i, sub_bits)
