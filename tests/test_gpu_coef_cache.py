"""Lanczos tables cached across batches (context option coef_cache_mb;
VERDICT r4 item 6), and WebDataset members submitted straight from a tar
shard resident in HBM (dg_wds_index offsets, the configs[2] bench path).

A pass's i16 weights depend only on its (box, in/out size, taps): a later
batch with the same pass reads the tables an earlier one computed.  Outputs
are bit-exact against the oracle and against a context with the cache off."""
import numpy as np
import pytest

from datago_amd import _lib as L
from datago_amd import synth
from oracle import buckets as B
from oracle import oracle as O

pytestmark = pytest.mark.gpu

KW = dict(crop_and_resize=True, default_image_size=512, downsampling_ratio=16, min_aspect_ratio=0.5,
          max_aspect_ratio=2.0, decode_semantics=1)


def _oracle(data, size=512, ratio=16):
    t = B.ARAwareTransform(size, ratio, 0.5, 2.0)
    with O.semantics(O.SEM_ZUNE):
        dec = O.jpeg_decode(data)[1]
    tw, th = t.target_size(dec.shape[1], dec.shape[0])
    return O.crop_and_resize(dec, tw, th, O.MODE_FIR) if (dec.shape[1], dec.shape[0]) != (tw, th) else dec


def test_cached_tables_bit_exact():
    datas = synth.mixed_corpus(91, 24, 200, 900)
    c = L.Context(0, **KW)
    first = c.decode_batch(datas)
    new0, hits0 = c.stat("coef_cache_new"), c.stat("coef_cache_hits")
    assert new0 > 0
    second = c.decode_batch(datas[::-1])  # every pass now reads cached tables
    assert c.stat("coef_cache_hits") - hits0 >= new0 // 2
    assert c.stat("coef_cache_new") == new0
    off = L.Context(0, **KW)
    off.set_option("coef_cache_mb", 0)
    plain = off.decode_batch(datas)
    for d, (s0, a0, _), (s1, a1, _), (s2, a2, _) in zip(datas, first, second[::-1], plain):
        assert s0 == s1 == s2 == 0
        assert np.array_equal(a0, a1) and np.array_equal(a0, a2)
    for d, (_, a, _) in list(zip(datas, first))[:6]:
        assert np.array_equal(a, _oracle(d))
    assert off.stat("coef_cache_new") == 0
    off.close()
    c.close()


def test_cache_arena_resets():
    """A 1 MiB arena fills within a few batches and starts over (after the
    batches reading it finish); outputs stay exact throughout."""
    c = L.Context(0, **KW)
    c.set_option("coef_cache_mb", 1)
    ref = L.Context(0, **KW)
    ref.set_option("coef_cache_mb", 0)
    for seed in (200, 201, 200, 202, 203, 204, 203, 205, 206, 205):  # repeats hit, new corpora fill the arena
        datas = synth.mixed_corpus(seed, 10, 300, 1400)
        tk = [c.submit_host(datas, [np.zeros(max(c.output_size(d)[1], 1), np.uint8) for d in datas])]
        got = c.decode_batch(datas)
        want = ref.decode_batch(datas)
        for (s0, a0, _), (s1, a1, _) in zip(got, want):
            assert s0 == s1 == 0 and np.array_equal(a0, a1)
        for t, metas, keep in tk:
            c.wait(t)
    assert c.stat("coef_cache_resets") > 0
    assert c.stat("coef_cache_hits") > 0
    c.close()
    ref.close()


def test_wds_members_from_shard_in_hbm():
    """configs[2]'s path: a shard uploaded once, its .jpg members submitted by
    their dg_wds_index offsets (no host copy of any member), bit-exact."""
    tars = [synth.make_wds_shard(300 + k, 24, first_key=100 * k) for k in range(2)]
    c = L.Context(0, **KW)
    arena = np.frombuffer(b"".join(tars) + bytes(64), np.uint8)
    d_arena = c.alloc(arena.nbytes)
    c.h2d(d_arena, arena)
    members, base = [], 0
    for t in tars:
        for smp in L.wds_index(t, 0, 1, "jpg"):
            members += [(base + off, n) for (name, off, n) in smp if name.endswith(".jpg")]
        base += len(t)
    assert len(members) == 48
    datas = [arena[off:off + n].tobytes() for off, n in members]
    sizes = [c.output_size(d)[1] for d in datas]
    outs = [c.alloc(s) for s in sizes]
    h_base = arena.ctypes.data
    tk, metas = c.submit_device([h_base + off for off, _ in members], [d_arena + off for off, _ in members],
                                [n for _, n in members], outs, sizes)
    c.wait(tk)
    for i, (d, s) in enumerate(zip(datas, sizes)):
        assert metas[i].status == 0
        got = np.empty(s, np.uint8)
        c.d2h(got, outs[i])
        assert np.array_equal(got, _oracle(d).reshape(-1)), i
    for p in outs:
        c.free(p)
    c.free(d_arena)
    c.close()
