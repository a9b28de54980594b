"""Host-out path into page-locked caller memory (dg_host_register): outputs
whose buffer lies in a registered range are DMA'd straight from HBM, bypassing
the pinned staging buffer and the host copy.  Same bytes as the staged path
and the oracle; pipelined submits reuse the pool; decode_one into a
registered buffer; unregistering waits for copies in flight."""
import ctypes
import numpy as np
import pytest

from datago_amd import synth
from oracle import buckets as B
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def test_registered_pool_direct_dma_bit_exact():
    from datago_amd import _lib as L
    ctx = L.Context(0, crop_and_resize=True, default_image_size=512, downsampling_ratio=16, min_aspect_ratio=0.5,
                    max_aspect_ratio=2.0)
    tr = B.ARAwareTransform(512, 16, 0.5, 2.0)
    datas = synth.mixed_corpus(21, 12, 96, 700)
    datas.append(synth.make_png(2101, 333, 222, "RGBA"))
    sizes = [ctx.output_size(d)[1] for d in datas]
    pools = [np.zeros(sum((n + 15) // 16 * 16 for n in sizes), np.uint8) for _ in range(2)]
    for p in pools:
        ctx.host_register(p)
    try:
        pend = []
        for k in range(4):  # two pools in turn, two batches in flight
            pool, o, outs = pools[k % 2], 0, []
            for n in sizes:
                outs.append(pool[o:o + n])
                o += (n + 15) // 16 * 16
            if len(pend) == 2:
                tk, metas, keep, outs0 = pend.pop(0)
                ctx.wait(tk)
            pend.append((*ctx.submit_host(datas, outs), outs))
        d0 = ctx.stat("direct_d2h")
        for tk, metas, keep, outs in pend:
            ctx.wait(tk)
            for i, (d, m, buf) in enumerate(zip(datas, metas, outs)):
                assert m.status == 0, i
                st, ref = O.decode_any(d)
                ref = O.crop_and_resize(ref, *tr.target_size(ref.shape[1], ref.shape[0]), O.MODE_FIR)
                assert np.array_equal(buf[: m.nbytes], ref.reshape(-1)), i
        assert ctx.stat("direct_d2h") >= len(datas) * 3  # every output of the registered pools went by DMA
        staged = ctx.decode_batch(datas)  # fresh (pageable) arrays: the staged path, same bytes
        for (st, arr, m), buf in zip(staged, pend[-1][3]):
            assert st == 0 and np.array_equal(arr.reshape(-1), buf[: m.nbytes])
        one = np.zeros(max(sizes), np.uint8)
        ctx.host_register(one)
        st, arr, m = ctx.decode_one(datas[0], out=one)
        assert st == 0 and np.array_equal(arr.reshape(-1), staged[0][1].reshape(-1))
        ctx.host_unregister(one)
        # a caller's buffer too small: the library says so (SMALL_BUFFER, size in the meta), the wrapper retries
        st, arr, m = ctx.decode_one(datas[0], out=np.zeros(16, np.uint8))
        assert st == 0 and np.array_equal(arr.reshape(-1), staged[0][1].reshape(-1))
        m = L.PayloadMeta()
        st = L.load().dg_decode_one(ctx._h, datas[0], len(datas[0]), -1, np.zeros(16, np.uint8).ctypes.data, 16,
                                    ctypes.byref(m))
        assert st == L.DG_ERR_SMALL_BUFFER and m.nbytes == staged[0][1].nbytes
    finally:
        for p in pools:
            ctx.host_unregister(p)
