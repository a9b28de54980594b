"""The oracle's JPEG decode-semantics switch (one switch
for the reference crates' unverifiable behaviour).

SEM_LIBJPEG is pinned bit-exactly to PIL / libjpeg-turbo (test_oracle_jpeg.py).
SEM_ZUNE restates zune-jpeg 0.5.12 -- the reference's decoder
(worker_files.rs:14-16 -> image 0.25.9 -> zune-jpeg) -- from its published
source; the crate is not vendored and no Rust toolchain exists here, so that
mode is PARITY UNPINNED.  What these tests pin is the stated per-channel
tolerance between the two (profiles/r02/semantics_envelope.json):
interior pixels within 8 LSB, p99 within 2, mean within 1; the last row and
column (where zune reads the MCU padding instead of replicating the edge)
within 48.
"""
import numpy as np
import pytest

from datago_amd import synth
from oracle import oracle as O


@pytest.fixture(scope="module")
def pairs():
    out = []
    for d in synth.mixed_corpus(31, 24, 64, 512):
        st, a = O.jpeg_decode(d)
        with O.semantics(O.SEM_ZUNE):
            st2, z = O.jpeg_decode(d)
        assert st == 0 and st2 == 0
        out.append((a.astype(np.int32), z.astype(np.int32)))
    return out


def test_switch_restores_default():
    d = synth.make_jpeg(1, 97, 61, 80, "4:2:0")
    a = O.jpeg_decode(d)[1]
    with O.semantics(O.SEM_ZUNE):
        pass
    assert np.array_equal(O.jpeg_decode(d)[1], a)


def test_modes_share_geometry_and_gray_paths(pairs):
    for a, z in pairs:
        assert a.shape == z.shape


def test_zune_envelope_per_channel(pairs):
    inner = np.concatenate([np.abs(a - z)[:-1, :-1].reshape(-1, a.shape[2]) for a, z in pairs if a.shape[2] == 3])
    edge = max(int(np.abs(a - z).max()) for a, z in pairs)
    assert inner.max() <= 8
    assert all(np.percentile(inner[:, c], 99) <= 2 for c in range(3))
    assert inner.mean(axis=0).max() <= 1.0
    assert edge <= 48


def test_zune_idct_differs_only_in_rounding():
    # a flat block decodes to the same level in both IDCTs (DC-only: both round (dc + 4) / 8)
    from PIL import Image
    import io
    for level in (0, 17, 128, 200, 255):
        buf = io.BytesIO()
        Image.fromarray(np.full((16, 16), level, np.uint8)).save(buf, format="JPEG", quality=95)
        a = O.jpeg_decode(buf.getvalue())[1]
        with O.semantics(O.SEM_ZUNE):
            z = O.jpeg_decode(buf.getvalue())[1]
        assert np.array_equal(a, z)
