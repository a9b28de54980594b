"""GPU parity for the PNG path (k_png_* kernels through the C ABI) against the
oracle (oracle/png_oracle.c, pinned to PIL by tests/test_oracle_png.py).
Tolerance 0 everywhere: inflate/unfilter/expand are exact by spec, the
resize is the same integer arithmetic as the JPEG path, alpha mul/div and the
f32 compositing are restated bit for bit."""
import hashlib
import json
import os
import zlib

import numpy as np
import pytest

from datago_amd import synth
from oracle import buckets as B
from oracle import oracle as O

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")


def _lib():
    from datago_amd import _lib as L
    return L


@pytest.fixture(scope="module")
def ctx_dec():
    return _lib().Context(0)


@pytest.fixture(scope="module")
def ctx_rgb8():
    return _lib().Context(0, image_to_rgb8=True)


@pytest.fixture(scope="module")
def ctx512():
    return _lib().Context(0, crop_and_resize=True, default_image_size=512, downsampling_ratio=16,
                          min_aspect_ratio=0.5, max_aspect_ratio=2.0)


@pytest.fixture(scope="module")
def ctx512_rgb8():
    return _lib().Context(0, crop_and_resize=True, default_image_size=512, downsampling_ratio=16,
                          min_aspect_ratio=0.5, max_aspect_ratio=2.0, image_to_rgb8=True)


def _cases():
    out = []
    i = 0
    for kind in synth.PNG_KINDS:
        for (w, h) in [(1, 1), (5, 3), (64, 33), (255, 7), (130, 300)]:
            for kw in ({}, {"level": 0}, {"strategy": zlib.Z_FIXED}, {"idat_max": 97, "level": 9}, {"filters": "4"}):
                i += 1
                if i % 2:
                    out.append((kind, w, h, kw))
    return out


CASES = _cases()


def _png(case):
    kind, w, h, kw = case
    return synth.make_png(hash((kind, w, h, str(kw))) & 0xFFFF, w, h, kind, **kw)


def test_png_decode_only_bit_exact(ctx_dec):
    datas = [_png(c) for c in CASES]
    res = ctx_dec.decode_batch(datas)
    for c, d, (st, arr, m) in zip(CASES, datas, res):
        ost, ref = O.png_decode(d)
        assert ost == 0
        assert st == 0, (c, st, _lib().last_error())
        assert arr.shape == ref.shape, c
        assert np.array_equal(arr, ref), (c, int(np.argwhere(arr != ref)[0][0]))
        assert (m.original_width, m.original_height, m.channels, m.bit_depth) == (ref.shape[1], ref.shape[0],
                                                                                 ref.shape[2], 8)


def test_png_golden_fixtures(ctx_dec):
    exp = json.load(open(os.path.join(GOLD, "png_expected.json")))
    names = sorted(exp)
    datas = [open(os.path.join(GOLD, "png", n + ".png"), "rb").read() for n in names]
    res = ctx_dec.decode_batch(datas)
    for n, (st, arr, m) in zip(names, res):
        assert st == exp[n]["status"], (n, st)
        if st == 0:
            assert list(arr.shape) == exp[n]["shape"], n
            assert hashlib.sha256(arr.tobytes()).hexdigest() == exp[n]["sha256"], n


def test_png_bucket_resize_bit_exact(ctx512):
    t = B.ARAwareTransform(512, 16, 0.5, 2.0)
    rng = np.random.default_rng(11)
    datas, kinds = [], []
    for i in range(36):
        kind = synth.PNG_KINDS[i % len(synth.PNG_KINDS)]
        w, h = int(rng.integers(20, 900)), int(rng.integers(20, 900))
        datas.append(synth.make_png(500 + i, w, h, kind, idat_max=int(rng.integers(0, 3)) * 8192))
        kinds.append((kind, w, h))
    res = ctx512.decode_batch(datas)
    for k, d, (st, arr, m) in zip(kinds, datas, res):
        assert st == 0, (k, st)
        _, ref = O.png_decode(d)
        tw, th = t.target_size(ref.shape[1], ref.shape[0])
        exp = O.crop_and_resize(ref, tw, th, O.MODE_FIR)
        assert arr.shape == exp.shape, k
        diff = np.argwhere(arr != exp)
        assert diff.size == 0, (k, diff[:3].tolist(), arr[tuple(diff[0])], exp[tuple(diff[0])])


def test_png_rgb8_conversions(ctx512_rgb8, ctx_rgb8):
    t = B.ARAwareTransform(512, 16, 0.5, 2.0)
    datas = [synth.make_png(900 + i, w, h, kind) for i, (kind, w, h) in enumerate(
        [("RGBA", 200, 150), ("LA", 151, 233), ("L", 90, 300), ("RGB", 640, 480), ("P8T", 120, 70),
         ("RGBA", 592, 432), ("LA", 592, 432)])]
    for ctx, resize in ((ctx512_rgb8, True), (ctx_rgb8, False)):
        res = ctx.decode_batch(datas)
        for d, (st, arr, m) in zip(datas, res):
            assert st == 0
            _, dec = O.png_decode(d)
            if resize:
                tw, th = t.target_size(dec.shape[1], dec.shape[0])
                resized = (tw, th) != (dec.shape[1], dec.shape[0])
                tr = O.crop_and_resize(dec, tw, th, O.MODE_FIR) if resized else dec
            else:
                resized, tr = False, dec
            exp = O.to_rgb8(tr, resized)
            assert m.channels == 3 and arr.shape == exp.shape
            assert np.array_equal(arr, exp), (dec.shape, resized)


def test_reference_rgba_composite_known_answers(ctx_rgb8):
    # worker_files.rs:322-383: 3x1 RGBA PNG through image_payload_from_path with img_to_rgb8
    rgba = np.array([[[255, 100, 50, 255], [200, 100, 50, 128], [255, 0, 0, 0]]], np.uint8)
    (st, arr, m), = ctx_rgb8.decode_batch([synth.pil_png(rgba)])
    assert st == 0 and (m.channels, m.bit_depth, m.width, m.height) == (3, 8, 3, 1)
    px = arr.reshape(-1).tolist()
    assert px[0:3] == [255, 100, 50]
    assert abs(px[3] - 164) <= 2 and abs(px[4] - 114) <= 2 and abs(px[5] - 89) <= 2
    assert px[6:9] == [128, 128, 128]
    # worker_files.rs:385-444: gray -> replicated, RGB passthrough
    (st, arr, m), = ctx_rgb8.decode_batch([synth.pil_png(np.array([[100]], np.uint8))])
    assert st == 0 and m.channels == 3 and arr.reshape(-1).tolist() == [100, 100, 100]
    (st, arr, m), = ctx_rgb8.decode_batch([synth.pil_png(np.array([[[255, 100, 50]]], np.uint8))])
    assert st == 0 and arr.reshape(-1).tolist() == [255, 100, 50]


def test_png_status_codes(ctx_dec):
    L = _lib()
    exp = json.load(open(os.path.join(GOLD, "png_expected.json")))
    bad = [n for n in sorted(exp) if exp[n]["status"]]
    datas = [open(os.path.join(GOLD, "png", n + ".png"), "rb").read() for n in bad]
    # corrupt inside the zlib stream (header intact): flipped bits in the IDAT payload
    good = bytearray(synth.make_png(77, 64, 64, "RGB"))
    i = good.index(b"IDAT") + 4
    for k in range(i + 2, min(i + 40, len(good) - 16)):
        good[k] ^= 0x5A
    datas.append(bytes(good))
    res = ctx_dec.decode_batch(datas)
    for n, (st, _, _) in zip(bad, res):
        assert st == exp[n]["status"], n
    assert res[-1][0] in (L.DG_ERR_CORRUPT, L.DG_OK)  # the oracle decides which
    assert res[-1][0] == (L.DG_OK if O.png_decode(bytes(good))[0] == 0 else L.DG_ERR_CORRUPT)


def test_mixed_jpeg_png_batch(ctx512):
    t = B.ARAwareTransform(512, 16, 0.5, 2.0)
    datas = []
    for i in range(12):
        if i % 2:
            datas.append(synth.make_png(300 + i, 100 + 37 * i, 80 + 29 * i, ["RGB", "L", "RGBA", "P8"][i % 4]))
        else:
            datas.append(synth.make_jpeg(300 + i, 100 + 37 * i, 80 + 29 * i, 90, "4:2:0"))
    res = ctx512.decode_batch(datas)
    for d, (st, arr, m) in zip(datas, res):
        assert st == 0
        _, dec = O.decode_any(d)
        tw, th = t.target_size(dec.shape[1], dec.shape[0])
        assert np.array_equal(arr, O.crop_and_resize(dec, tw, th, O.MODE_FIR))


def test_png_large_full_size_properties(ctx512):
    # bench-sized PNG: decode equals the oracle; resize output has the bucket's dims
    d = synth.make_png(4242, 1800, 1200, "RGB")
    (st, arr, m), = _lib().Context(0).decode_batch([d])
    assert st == 0
    _, ref = O.png_decode(d)
    assert np.array_equal(arr, ref)
    (st, arr, m), = ctx512.decode_batch([d])
    t = B.ARAwareTransform(512, 16, 0.5, 2.0)
    assert st == 0 and (arr.shape[1], arr.shape[0]) == t.target_size(1800, 1200)


@pytest.mark.parametrize("inf_decode,inf_chunk,stage3",
                         [(d, 32768, 32) for d in range(29) if d != 10] +
                         [(2, 4096, 32), (2, 8192, 32), (2, 16384, 32), (3, 65536, 32), (9, 16384, 32)] +
                         [(25, 32768, s) for s in (8, 16, 64)])
def test_chunked_inflate_matches_serial_and_oracle(inf_decode, inf_chunk, stage3):
    """Large streams take the chunk-parallel inflate (block-header search,
    one lane per chunk, window markers); it must equal the oracle and the
    serial kernel (option png_chunked=0) byte for byte, for every
    k_inf_decode shape (option inf_decode: lanes per workgroup, lookup bits)
    and chunk size (option inf_chunk: compressed bytes per chunk), and the
    block finder's round size (option inf_stage3)."""
    L = _lib()
    rng = np.random.default_rng(31)
    datas = []
    for i, (w, h) in enumerate([(1500, 1000), (700, 2100), (2048, 600), (999, 777)]):
        px = synth.synth_pixels(rng, w, h)
        if i == 1:  # flat graphics: highly compressible, long matches
            px = (px // 64) * 64
        datas.append(synth.pil_png(px, compress_level=[6, 9, 1, 6][i]))
    datas.append(synth.make_png(77, 1200, 900, "RGBA", level=6))
    datas.append(synth.make_png(78, 1600, 1000, "L", level=6, filters="random"))
    a = L.Context(0)
    a.set_option("inf_decode", inf_decode)
    a.set_option("inf_chunk", inf_chunk)
    a.set_option("inf_stage3", stage3)
    b = L.Context(0)
    b.set_option("png_chunked", 0)
    ra, rb = a.decode_batch(datas), b.decode_batch(datas)
    for d, (sa, xa, _), (sb, xb, _) in zip(datas, ra, rb):
        _, ref = O.png_decode(d)
        assert sa == 0 and sb == 0
        assert np.array_equal(xa, ref) and np.array_equal(xb, ref)
    assert a.stat("png_chunks") > 0
    print("chunks", a.stat("png_chunks"), "serial fallbacks", a.stat("png_serial_fallbacks"))
    if inf_chunk >= 32768:  # the finder found every chunk's block start (a miss would only cost speed)
        assert a.stat("png_serial_fallbacks") == 0


A7_CASES = [(k, w, h) for k in synth.PNG_KINDS for (w, h) in [(1, 1), (2, 3), (5, 9), (8, 8), (33, 17), (257, 130)]]


def test_png_adam7_bit_exact(ctx_dec, ctx512):
    """Adam7-interlaced PNGs (PNG spec 8.2): seven passes inflated together,
    each unfiltered as its own sub-image, scattered by k_png_expand; tiny
    sizes leave passes empty.  Oracle pinned vs PIL (test_oracle_png)."""
    datas = [synth.make_png(hash((k, w, h, "a7")) & 0xFFFF, w, h, k, interlace=True) for (k, w, h) in A7_CASES]
    for c, d, (st, arr, m) in zip(A7_CASES, datas, ctx_dec.decode_batch(datas)):
        ost, ref = O.png_decode(d)
        assert ost == 0 and st == 0, (c, st, _lib().last_error())
        assert arr.shape == ref.shape and np.array_equal(arr, ref), c
    # large (chunk-parallel inflate) and resized
    t = B.ARAwareTransform(512, 16, 0.5, 2.0)
    big = [synth.make_png(61, 1400, 900, "RGB", interlace=True), synth.make_png(62, 700, 1300, "RGBA", interlace=True),
           synth.make_png(63, 1000, 1000, "P4", interlace=True)]
    for d, (st, arr, m) in zip(big, ctx512.decode_batch(big)):
        assert st == 0
        _, ref = O.png_decode(d)
        tw, th = t.target_size(ref.shape[1], ref.shape[0])
        assert np.array_equal(arr, O.crop_and_resize(ref, tw, th, O.MODE_FIR))


@pytest.mark.parametrize("uf_units", [2, 1])
def test_serial_inflate_beside_chunked_and_unfilter_unit_widths(uf_units):
    """Round-2 scheduling paths: small streams (masks) inflate on the side
    stream beside the chunk-parallel kernels (option side_stream 1, mode 0 +
    fallbacks mode 1) or after them on the main stream (side_stream 0, mode
    2); and the pipelined unfilter sizes its LDS for the batch's widest filter
    unit (L-only batches: 6 workers per CU, RGBA: 1).  Every variant equals
    the oracle byte for byte; tall images give many pipelined bands.  Both
    unfilter tile widths (option uf_units: 64 or 128 filter units) run."""
    L = _lib()
    rng = np.random.default_rng(47)
    big = [synth.pil_png(synth.synth_pixels(rng, 1300, 1700), compress_level=6),  # chunked
           synth.make_png(90, 900, 2300, "RGBA", level=6)]
    small = [synth.make_png(91 + i, 300 + 50 * i, 900 + 31 * i, "L", level=9) for i in range(3)]  # serial
    batches = {"mixed": big + small, "L_only": small + [synth.make_png(95, 640, 2600, "L", level=6)],
               "RGBA_only": [big[1], synth.make_png(96, 333, 1111, "RGBA", level=1)]}
    for side in (1, 0):
        ctx = L.Context(0)
        ctx.set_option("side_stream", side)
        ctx.set_option("uf_units", uf_units)
        for name, datas in batches.items():
            for k, (d, (st, arr, _)) in enumerate(zip(datas, ctx.decode_batch(datas))):
                ost, ref = O.png_decode(d)
                assert ost == 0 and st == 0, (side, name, k, st, L.last_error())
                assert arr.shape == ref.shape and np.array_equal(arr, ref), (side, name, k)


DBG_FORCE_UF_TIMEOUT = 1 << 18


def test_unfilter_wait_timeout_is_unsupported_not_corrupt():
    """A band whose wait for the previous band times out (a starved producer,
    e.g. ranks sharing the GPU) returns the image DG_ERR_UNSUPPORTED -- valid
    data the caller's CPU decoder takes -- not DG_ERR_CORRUPT, which would drop
    the sample.  Test switch: band 1 of every plane times out on its first
    wait.  Images of one band (<= 64 rows) never wait and stay bit-exact; the
    kernel returns (no hang)."""
    L = _lib()
    ctx = L.Context(0)
    tall = [synth.make_png(1301, 200, 130, "RGB"), synth.make_png(1302, 90, 700, "L", level=6)]
    short = [synth.make_png(1303, 300, 64, "RGBA"), synth.make_png(1304, 50, 20, "P8")]
    ctx.set_option("debug_flags", DBG_FORCE_UF_TIMEOUT)
    try:
        res = ctx.decode_batch(tall + short)
    finally:
        ctx.set_option("debug_flags", 0)
    for st, _, _ in res[:2]:
        assert st == L.DG_ERR_UNSUPPORTED
    for d, (st, arr, _) in zip(short, res[2:]):
        assert st == 0
        ost, ref = O.png_decode(d)
        assert np.array_equal(arr.reshape(ref.shape), ref)
    for d, (st, arr, _) in zip(tall, ctx.decode_batch(tall)):  # switch off: decoded again
        assert st == 0
        assert np.array_equal(arr.reshape(O.png_decode(d)[1].shape), O.png_decode(d)[1])


def test_many_serial_fallbacks_bit_exact_and_timed():
    """streams the chunked inflate cannot start in (zlib level 0 =
    stored blocks, Z_FIXED = fixed-Huffman blocks: the block finder looks for
    dynamic-Huffman headers) fall back to the serial kernel, which now claims
    images from a work counter on up to one workgroup per CU instead of 4
    fixed workgroups walking the list.  Every image bit-exact; the batch's
    time is printed (tools/gpu_png.sh: compare before / after)."""
    import time
    L = _lib()
    rng = np.random.default_rng(41)
    datas = []
    for i in range(48):
        px = synth.synth_pixels(rng, 300 + 7 * i, 260 + 5 * i)
        datas.append(synth.pil_png(px, compress_level=0) if i % 2 == 0 else
                     synth.make_png(500 + i, 300 + 7 * i, 260 + 5 * i, "RGB", strategy=zlib.Z_FIXED))
    a = L.Context(0)
    a.decode_batch(datas[:2])
    f0 = a.stat("png_serial_fallbacks")
    t0 = time.perf_counter()
    ra = a.decode_batch(datas)
    dt = time.perf_counter() - t0
    nfb = a.stat("png_serial_fallbacks") - f0
    print(f"{len(datas)} images, {nfb} serial fallbacks, {dt * 1e3:.1f} ms")
    for d, (sa, xa, _) in zip(datas, ra):
        _, ref = O.png_decode(d)
        assert sa == 0 and np.array_equal(xa, ref)
    assert nfb + a.stat("png_small_streams") > 0


@pytest.mark.parametrize("inf_cap,inf_pad", [(10, 65536), (15, 65536), (20, 65536), (15, 4096), (10, 0)])
def test_chunk_entry_capacity_bit_exact(inf_cap, inf_pad):
    """Option inf_cap (the chunk-parallel inflate's entries per chunk, in tenths
    of the image's expansion of a span; VERDICT r5 item 5: the entries were
    most of a PNG batch's device memory).  A chunk that outgrows its entries
    sends its image to the serial kernel: smaller capacities stay bit-exact."""
    L = _lib()
    rng = np.random.default_rng(33)
    datas = []
    for i, (w, h) in enumerate([(1500, 1000), (700, 2100), (2048, 600)]):
        px = synth.synth_pixels(rng, w, h)
        if i == 1:
            px = (px // 64) * 64  # flat regions: the expansion varies along the stream
        datas.append(synth.pil_png(px, compress_level=6))
    datas.append(synth.make_png(79, 1200, 900, "RGBA", level=6))
    a = L.Context(0)
    a.set_option("inf_cap", inf_cap)
    a.set_option("inf_pad", inf_pad)
    for d, (sa, xa, _) in zip(datas, a.decode_batch(datas)):
        _, ref = O.png_decode(d)
        assert sa == 0 and np.array_equal(xa, ref)
    print("inf_cap", inf_cap, "chunks", a.stat("png_chunks"), "serial fallbacks", a.stat("png_serial_fallbacks"))
