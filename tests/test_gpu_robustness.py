"""Real-world JPEG robustness on the GPU.

* Baseline JPEGs with per-image optimised Huffman tables (PIL optimize=True,
  as mozjpeg / web corpora) and with deliberately deep tables (10- and 16-bit
  codes over more 9-bit prefixes than the decoder has sub-tables: the lim[]
  fallback of build_huff_table), bit-exact against the oracle -- which is
  itself checked against PIL (libjpeg-turbo) here.  The reference decodes all
  of them (worker_files.rs:8-17 -> zune-jpeg).
* The Huffman/quantisation table pools never turn a valid image into an error,
  however many distinct tables one context sees (> 65,535 here).
* Entropy-decode failures the host cannot rule out (a write pass that leaves a
  range in another state than the sync pass, a boundary repair that does not
  settle) come back as a per-image DG_ERR_UNSUPPORTED -- the caller's CPU
  decoder takes the image -- never as DG_OK with wrong pixels.  Forced with
  the context's debug switches.
"""
import ctypes
import io

import numpy as np
import pytest
from PIL import Image

from datago_amd import synth
from oracle import buckets as B
from oracle import oracle as O

pytestmark = pytest.mark.gpu

DBG_FORCE_WRITE_MISMATCH = 1 << 16
DBG_FORCE_CHAIN_CHANGE = 1 << 17


def _lib():
    from datago_amd import _lib as L
    return L


def _pil(data, gray):
    return np.asarray(Image.open(io.BytesIO(data)).convert("L" if gray else "RGB"))


def _optimised_corpus():
    """(bytes, gray) pairs: PIL optimize=True at low and high quality (the
    low-quality noisy images give the deepest optimal trees), plus the
    custom-table encoder with optimal and deep tables, with and without
    restart intervals."""
    out = []
    for i in range(12):
        rng = np.random.default_rng(9100 + i)
        w, h = int(rng.integers(24, 520)), int(rng.integers(24, 520))
        gray = i % 6 == 5
        arr = synth.synth_pixels(rng, w, h, gray)
        if i % 3 == 0:  # high-entropy content: long codes in the optimal tables
            arr = rng.integers(0, 256, arr.shape, dtype=np.uint8)
        buf = io.BytesIO()
        # (noise at high quality outgrows PIL's single-buffer optimize pass)
        kw = dict(quality=30 if i % 3 == 0 else [15, 50, 80, 97][i % 4], optimize=True)
        if not gray:
            kw["subsampling"] = [0, 1, 2][i % 3]
        Image.fromarray(arr).save(buf, format="JPEG", **kw)
        out.append((buf.getvalue(), gray))
    for i, (tables, ss, gray, rst) in enumerate([("optimal", "4:2:0", False, 0), ("optimal", "4:4:4", False, 2),
                                                 ("optimal", "4:2:0", True, 0), ("deep", "4:2:0", False, 0),
                                                 ("deep", "4:4:4", False, 0), ("deep", "4:2:0", True, 0),
                                                 ("deep", "4:2:0", False, 3), ("deep", "4:4:4", False, 1)]):
        rng = np.random.default_rng(9200 + i)
        w, h = int(rng.integers(16, 400)), int(rng.integers(16, 400))
        arr = synth.synth_pixels(rng, w, h, gray)
        if i % 2:
            arr = rng.integers(0, 256, arr.shape, dtype=np.uint8)
        out.append((synth.encode_jpeg_tables(arr, [30, 75, 95][i % 3], ss, tables, restart_interval=rst), gray))
    return out


@pytest.fixture(scope="module")
def corpus():
    return _optimised_corpus()


def test_corpus_exercises_long_codes(corpus):
    """The fixtures really contain >9-bit codes, and the deep ones more long
    9-bit prefixes than the decoder has sub-tables (kMaxSubTables = 8)."""
    deep_prefixes = []
    for data, _ in corpus:
        i = 2
        while i < len(data) - 4:
            if data[i] == 0xFF and data[i + 1] == 0xC4:
                seg = data[i + 4:i + 2 + int.from_bytes(data[i + 2:i + 4], "big")]
                j = 0
                while j < len(seg):
                    bits = list(seg[j + 1:j + 17])
                    code, prefixes = 0, set()
                    for L_, n in enumerate(bits, start=1):
                        for _ in range(n):
                            if L_ > 9:
                                prefixes.add(code >> (L_ - 9))
                            code += 1
                        code <<= 1
                    deep_prefixes.append(len(prefixes))
                    j += 17 + sum(bits)
            if data[i] == 0xFF and data[i + 1] == 0xDA:
                break
            i += 1
    assert max(deep_prefixes) > 8, deep_prefixes
    assert sum(1 for p in deep_prefixes if p > 0) >= 8, deep_prefixes


def test_oracle_matches_pil_on_optimised_tables(corpus):
    for data, gray in corpus:
        st, dec = O.jpeg_decode(data)
        assert st == 0
        d = dec[:, :, 0] if gray and dec.ndim == 3 else dec
        assert np.array_equal(d, _pil(data, gray))


def test_optimised_and_deep_tables_decode_bit_exact(corpus):
    ctx = _lib().Context(0)
    res = ctx.decode_batch([d for d, _ in corpus])
    for k, ((data, gray), (st, arr, meta)) in enumerate(zip(corpus, res)):
        assert st == 0, (k, st, _lib().last_error())
        _, dec = O.jpeg_decode(data)
        assert arr.shape == dec.shape and np.array_equal(arr, dec), k
    assert ctx.stat("write_mismatch") == 0


@pytest.mark.parametrize("sub_bits", [0, 256])
def test_optimised_tables_crop_resize_bit_exact(corpus, sub_bits):
    ctx = _lib().Context(0, crop_and_resize=True, default_image_size=512, downsampling_ratio=16,
                         min_aspect_ratio=0.5, max_aspect_ratio=2.0)
    if sub_bits:  # many short subsequences: every long-code path crosses subsequence boundaries
        ctx.set_option("sub_bits", sub_bits)
    t = B.ARAwareTransform(512, 16, 0.5, 2.0)
    res = ctx.decode_batch([d for d, _ in corpus])
    for k, ((data, gray), (st, arr, meta)) in enumerate(zip(corpus, res)):
        assert st == 0, (k, st)
        _, dec = O.jpeg_decode(data)
        tw, th = t.target_size(dec.shape[1], dec.shape[0])
        ref = O.crop_and_resize(dec, tw, th, O.MODE_FIR)
        assert np.array_equal(arr, ref), k


def _patched_quant_jpegs(n):
    """n gray 16x16 JPEGs, each with its own quantisation table (the last
    three zigzag entries encode the index): n distinct pool entries."""
    rng = np.random.default_rng(77)
    buf = io.BytesIO()
    Image.fromarray(synth.synth_pixels(rng, 16, 16, True)).save(buf, format="JPEG", quality=50)
    base = bytearray(buf.getvalue())
    dqt = base.index(b"\xff\xdb")
    assert base[dqt + 4] == 0  # one 8-bit table, id 0
    q0 = dqt + 5
    out = []
    for i in range(n):
        b = bytearray(base)
        b[q0 + 61] = 1 + i % 251
        b[q0 + 62] = 1 + (i // 251) % 251
        b[q0 + 63] = 1 + (i // (251 * 251)) % 251
        out.append(bytes(b))
    return out


def test_table_pools_never_fill():
    n = 70_000
    datas = _patched_quant_jpegs(n)
    L = _lib()
    ctx = L.Context(0)
    checks = list(range(0, n, 4999)) + [n - 1]
    want = {i: O.jpeg_decode(datas[i])[1] for i in checks}
    batch = 4096
    for lo in range(0, n, batch):
        res = ctx.decode_batch(datas[lo:lo + batch])
        bad = [(lo + j, r[0]) for j, r in enumerate(res) if r[0] != 0]
        assert not bad, (bad[:5], L.last_error())
        for i in checks:
            if lo <= i < lo + batch:
                assert np.array_equal(res[i - lo][1], want[i]), i
    assert ctx.stat("pool_flushes") >= 1
    assert ctx.stat("qpool") <= 16384 + batch  # kPoolKeep


def test_forced_write_mismatch_is_a_per_image_status():
    L = _lib()
    ctx = L.Context(0, crop_and_resize=True, default_image_size=512, downsampling_ratio=16,
                    min_aspect_ratio=0.5, max_aspect_ratio=2.0)
    jpgs = [synth.make_jpeg(500 + i, 300 + 40 * i, 200 + 30 * i, 85, "4:2:0") for i in range(3)]
    png = synth.make_png(7, 120, 90, "RGB")
    ctx.set_option("debug_flags", DBG_FORCE_WRITE_MISMATCH)
    res = ctx.decode_batch(jpgs + [png])
    assert [r[0] for r in res] == [L.DG_ERR_UNSUPPORTED] * 3 + [0]
    assert ctx.stat("write_mismatch") >= 3
    ctx.set_option("debug_flags", 0)
    res = ctx.decode_batch(jpgs)
    assert [r[0] for r in res] == [0] * 3
    t = B.ARAwareTransform(512, 16, 0.5, 2.0)
    for d, (st, arr, meta) in zip(jpgs, res):
        _, dec = O.jpeg_decode(d)
        assert np.array_equal(arr, O.crop_and_resize(dec, *t.target_size(dec.shape[1], dec.shape[0]), O.MODE_FIR))


def test_unsettled_resync_is_a_per_image_status():
    L = _lib()
    ctx = L.Context(0)
    jpgs = [synth.make_jpeg(600 + i, 256, 192, 90, "4:2:0") for i in range(2)]
    png = synth.make_png(8, 64, 48, "RGBA")
    ctx.set_option("debug_flags", DBG_FORCE_CHAIN_CHANGE)
    res = ctx.decode_batch(jpgs + [png])
    assert [r[0] for r in res] == [L.DG_ERR_UNSUPPORTED] * 2 + [0]
    assert ctx.stat("unsettled_batches") == 1
    assert np.array_equal(res[2][1], O.png_decode(png)[1])
    ctx.set_option("debug_flags", 0)
    res = ctx.decode_batch(jpgs)
    assert all(r[0] == 0 and np.array_equal(r[1], O.jpeg_decode(d)[1]) for d, r in zip(jpgs, res))


@pytest.mark.parametrize("key,value", [("inf_decode", 99), ("slots", 0), ("coalesce_max", 0), ("sub_bits", 100),
                                       ("decode_semantics", 2), ("no_such_option", 1)])
def test_rejected_option_names_itself_in_last_error(key, value):
    """a failing dg_ctx_set_option sets dg_last_error to a
    message naming the option, the value and the accepted range (a stale
    message from an earlier failure -- round 5's "truncated PNG chunk" after
    an out-of-range inf_decode -- must not survive)."""
    L = _lib()
    ctx = L.Context(0)
    ctx.set_option("slots", 4)
    h = ctypes.c_void_p()
    assert L.load().dg_bucket_table_build(224, 0, 0.5, 2.0, ctypes.byref(h)) == L.DG_ERR_INVALID  # a stale message
    assert L.load().dg_ctx_set_option(ctx._h, key.encode(), value) == L.DG_ERR_INVALID
    msg = L.last_error()
    assert key in msg and str(value) in msg, msg
    assert ("unknown option" in msg) if key == "no_such_option" else ("valid unless" in msg), msg
    assert L.load().dg_ctx_get_stat(ctx._h, b"no_such_stat") == -1
    assert "no_such_stat" in L.last_error()
    ctx.close()
