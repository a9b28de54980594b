"""Corrupt inputs on the GPU path: bit flips in entropy-coded / zlib data,
truncations, and damaged headers, mixed into batches with good images.  The
kernels must neither fault nor hang, good images in the same batch must stay
bit-exact, and every status must be one the reference maps (OK, CORRUPT,
UNSUPPORTED).  Where the oracle rejects a file the GPU must not report OK
with different pixels: either both decode (and agree) or the GPU reports an
error -- libjpeg-style recovery from bad Huffman codes is not reproduced, so
a corrupt scan the oracle happens to decode may come back CORRUPT."""
import numpy as np
import pytest

from datago_amd import synth
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _lib():
    from datago_amd import _lib as L
    return L


def _flip(data: bytes, rng, start: int, n: int) -> bytes:
    b = bytearray(data)
    for _ in range(n):
        i = int(rng.integers(start, len(b)))
        b[i] ^= 1 << int(rng.integers(0, 8))
    return bytes(b)


def _corpus(seed: int):
    rng = np.random.default_rng(seed)
    good, bad = [], []
    for i in range(12):
        w, h = int(rng.integers(16, 600)), int(rng.integers(16, 600))
        kind = i % 4
        if kind == 0:
            d = synth.make_jpeg(seed * 100 + i, w, h, int(rng.integers(50, 96)), ["4:2:0", "4:2:2", "4:4:4"][i % 3],
                                restart_marker_rows=int(rng.integers(0, 3)))
        elif kind == 1:
            d = synth.make_jpeg(seed * 100 + i, w, h, 85, progressive=True)
        elif kind == 2:
            d = synth.make_png(seed * 100 + i, w, h, synth.PNG_KINDS[i % len(synth.PNG_KINDS)])
        else:
            d = synth.make_png(seed * 100 + i, w, h, "RGB", interlace=True)
        good.append(d)
        n = len(d)
        # flips past the headers, a truncation, a flipped header byte
        bad.append(_flip(d, rng, min(n - 1, 700), int(rng.integers(1, 20))))
        bad.append(d[: int(rng.integers(n // 3, n - 1))])
        bad.append(_flip(d, rng, 2, 1))
    return good, bad


@pytest.mark.parametrize("seed", [1, 2, 3, 4])
def test_corrupt_inputs_do_not_fault(seed):
    L = _lib()
    ctx = L.Context(0, crop_and_resize=True, default_image_size=512, downsampling_ratio=16,
                    min_aspect_ratio=0.5, max_aspect_ratio=2.0)
    ctx.set_option("progressive", 1)
    good, bad = _corpus(seed)
    rng = np.random.default_rng(seed)
    order = rng.permutation(len(good) + len(bad))
    datas = [(good + bad)[k] for k in order]
    res = ctx.decode_batch(datas)
    ok_statuses = {L.DG_OK, L.DG_ERR_CORRUPT, L.DG_ERR_UNSUPPORTED}
    ref_ctx = L.Context(0, crop_and_resize=True, default_image_size=512, downsampling_ratio=16,
                        min_aspect_ratio=0.5, max_aspect_ratio=2.0)
    ref_ctx.set_option("progressive", 1)
    clean = ref_ctx.decode_batch(good)
    for k, d, (st, arr, meta) in zip(order, datas, res):
        assert st in ok_statuses, (k, st)
        if k < len(good):  # good images are unaffected by their corrupt neighbours
            assert st == L.DG_OK and np.array_equal(arr, clean[k][1]), k
    # the same batch again: no state leaks between batches
    res2 = ctx.decode_batch(datas)
    assert [r[0] for r in res2] == [r[0] for r in res]
