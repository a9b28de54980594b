"""Decode-semantics switch on the GPU (context option "decode_semantics").

0 (default): libjpeg-turbo semantics, the oracle's pinned mode.
1: zune-jpeg 0.5.12 -- the reference's own decoder (worker_files.rs:14-16 ->
image 0.25.9 -> zune-jpeg) -- restated in the oracle's SEM_ZUNE mode from the
crate's published source.  That restatement is PARITY UNPINNED (the crate is
not vendored); what is pinned here is that the GPU's zune mode
is bit-exact to it, so a toolchain that can run the crate can confirm or fix
one restatement and both paths follow.  Widths/heights around the MCU padding
exercise zune's edge handling (it reads the padded rows instead of
replicating the last sample)."""
import numpy as np
import pytest

from datago_amd import synth
from oracle import buckets as B
from oracle import oracle as O

pytestmark = pytest.mark.gpu

SIZES = [(64, 48), (65, 49), (63, 47), (62, 46), (16, 16), (17, 9), (1, 1), (2, 2), (3, 5), (130, 67), (333, 211),
         (1000, 10), (10, 700)]


def _corpus():
    out = []
    for i, (w, h) in enumerate(SIZES):
        for j, ss in enumerate(["4:2:0", "4:2:2", "4:4:4"]):
            out.append(synth.make_jpeg(7000 + 10 * i + j, w, h, [60, 85, 95][j], ss, gray=(i + j) % 5 == 4,
                                       restart_marker_rows=1 if (i + j) % 4 == 1 else 0))
    return out


@pytest.fixture(scope="module")
def corpus():
    return _corpus()


def _ctx(sem, resize):
    from datago_amd import _lib as L
    kw = dict(crop_and_resize=True, default_image_size=512, downsampling_ratio=16, min_aspect_ratio=0.5,
              max_aspect_ratio=2.0) if resize else {}
    c = L.Context(0, **kw)
    c.set_option("decode_semantics", sem)
    return c


def _oracle(d, sem):
    with O.semantics(sem):
        st, dec = O.jpeg_decode(d)
    assert st == 0
    return dec


def test_zune_decode_bit_exact_vs_restatement(corpus):
    res = _ctx(1, False).decode_batch(corpus)
    for k, (d, (st, arr, meta)) in enumerate(zip(corpus, res)):
        assert st == 0, k
        ref = _oracle(d, O.SEM_ZUNE)
        assert np.array_equal(arr, ref), (k, SIZES[k // 3])


def test_zune_crop_resize_bit_exact_vs_restatement(corpus):
    t = B.ARAwareTransform(512, 16, 0.5, 2.0)
    res = _ctx(1, True).decode_batch(corpus)
    for k, (d, (st, arr, meta)) in enumerate(zip(corpus, res)):
        assert st == 0, k
        dec = _oracle(d, O.SEM_ZUNE)
        ref = O.crop_and_resize(dec, *t.target_size(dec.shape[1], dec.shape[0]), O.MODE_FIR)
        assert np.array_equal(arr, ref), (k, SIZES[k // 3])


def test_default_semantics_unchanged_and_modes_differ(corpus):
    a = _ctx(0, False).decode_batch(corpus)
    z = _ctx(1, False).decode_batch(corpus)
    differ = 0
    for d, (sa, xa, _), (sz, xz, _) in zip(corpus, a, z):
        assert np.array_equal(xa, _oracle(d, O.SEM_LIBJPEG))
        differ += int(not np.array_equal(xa, xz))
    assert differ > len(corpus) // 2


def test_option_validated():
    from datago_amd import _lib as L
    c = L.Context(0)
    with pytest.raises(Exception):
        c.set_option("decode_semantics", 2)


def _truncate_scans(data: bytes, keep: int) -> bytes:
    """The progressive file cut after its first `keep` scans (+ EOI): valid,
    with coefficients left incompletely refined -- libjpeg would smooth those
    blocks (jdcoefct.c), zune-jpeg decodes them as they stand."""
    sos = [i for i in range(len(data) - 1) if data[i] == 0xFF and data[i + 1] == 0xDA]
    assert len(sos) > keep
    # the scan after `keep` starts at its SOS (or at a DHT just before it)
    cut = sos[keep]
    j = cut - 1
    while j > sos[keep - 1] and not (data[j] == 0xFF and data[j + 1] == 0xC4):
        j -= 1
    if j > sos[keep - 1]:
        cut = j
    return data[:cut] + b"\xff\xd9"


def test_incomplete_progressive_refinement_decodes_in_zune_mode():
    from datago_amd import _lib as L
    datas = [_truncate_scans(synth.make_jpeg(7400 + i, w, h, 88, ss, progressive=True), keep)
             for i, (w, h, ss, keep) in enumerate([(300, 200, "4:2:0", 3), (257, 131, "4:4:4", 5),
                                                    (640, 480, "4:2:0", 7), (99, 301, "4:2:2", 2)])]
    lj = _ctx(0, False)
    lj.set_option("progressive", 1)
    zu = L.Context(0, decode_semantics=1)  # through dg_image_config.decode_semantics
    zu.set_option("progressive", 1)
    for d, (st, _, _) in zip(datas, lj.decode_batch(datas)):
        assert st == L.DG_ERR_UNSUPPORTED  # libjpeg semantics would block-smooth
        assert O.jpeg_decode(d)[0] == O.OJ_UNSUPPORTED
    for k, (d, (st, arr, _)) in enumerate(zip(datas, zu.decode_batch(datas))):
        assert st == 0, (k, L.last_error())
        assert np.array_equal(arr, _oracle(d, O.SEM_ZUNE)), k


def test_zune_complete_progressive_full_size_1024():
    """Complete (not truncated) progressive files in zune mode, configs[1]
    sizes, decode + bucket + crop/resize at 1024/32 through the default split
    submission (the progressive aggregate), mixed with baseline files: every
    output bit-exact against the SEM_ZUNE oracle."""
    from datago_amd import _lib as L
    ctx = L.Context(0, crop_and_resize=True, default_image_size=1024, downsampling_ratio=32, min_aspect_ratio=0.5,
                    max_aspect_ratio=2.0, decode_semantics=1)
    dims = [(2048, 1536, "4:2:0", True), (1100, 1900, "4:2:2", True), (1500, 1500, "4:4:4", True),
            (1999, 1001, "4:2:0", False), (777, 1333, "4:2:0", True), (2300, 1100, "4:2:0", False)]
    datas = [synth.make_jpeg(7600 + i, w, h, 90, ss, gray=(i == 4), progressive=p) for i, (w, h, ss, p) in
             enumerate(dims)]
    t = B.ARAwareTransform(1024, 32, 0.5, 2.0)
    for k, (d, (st, arr, meta)) in enumerate(zip(datas, ctx.decode_batch(datas))):
        assert st == 0, (k, L.last_error())
        dec = _oracle(d, O.SEM_ZUNE)
        ref = O.crop_and_resize(dec, *t.target_size(dec.shape[1], dec.shape[0]), O.MODE_FIR)
        assert np.array_equal(arr, ref), (k, dims[k])
    assert ctx.stat("prog_aggregate_images") == sum(p for *_, p in dims)
