"""GPU parity for progressive JPEG (zune-jpeg decodes
"baseline + progressive"): k_prog_zero + k_prog_scan through the C ABI vs
the oracle's jdphuff.c restatement, bit-exact, and vs PIL/libjpeg-turbo.
Scripts are libjpeg's default progression (jpeg_simple_progression), which
is what PIL writes; sizes, samplings, gray, quality and restart intervals
vary."""
import io

import numpy as np
import pytest
from PIL import Image

from datago_amd import synth
from oracle import buckets as B
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _lib():
    from datago_amd import _lib as L
    return L


def _prog(seed, w, h, q=85, ss="4:2:0", gray=False, rst=0):
    rng = np.random.default_rng(seed)
    return synth.encode_jpeg(synth.synth_pixels(rng, w, h, gray), q, ss, restart_marker_blocks=rst, progressive=True)


def _cases(seed, n, maxdim):
    out = []
    for i in range(n):
        rng = np.random.default_rng(seed * 1000 + i)
        w, h = int(rng.integers(1, maxdim)), int(rng.integers(1, maxdim))
        out.append(_prog(seed * 1000 + i, w, h, int(rng.integers(20, 101)), ["4:2:0", "4:2:2", "4:4:4"][i % 3],
                         i % 7 == 6, int(rng.integers(1, 12)) if i % 4 == 1 else 0))
    return out


def test_progressive_decode_bit_exact():
    L = _lib()
    ctx = L.Context(0)
    ctx.set_option("progressive", 1)
    datas = _cases(31, 24, 500)
    for i, (data, (st, arr, meta)) in enumerate(zip(datas, ctx.decode_batch(datas))):
        assert st == 0, (i, L.last_error())
        ost, ref = O.jpeg_decode(data)
        assert ost == 0
        assert np.array_equal(arr.reshape(ref.shape), ref), i
        pil = np.asarray(Image.open(io.BytesIO(data)))
        assert np.array_equal(arr.reshape(pil.shape), pil), i


def test_progressive_mixed_with_baseline_and_resized():
    L = _lib()
    ctx = L.Context(0, crop_and_resize=True, default_image_size=512, downsampling_ratio=16,
                    min_aspect_ratio=0.5, max_aspect_ratio=2.0)
    ctx.set_option("progressive", 1)
    datas = []
    for i in range(8):
        datas.append(synth.make_jpeg(700 + i, 200 + 97 * i, 640 - 53 * i, 80 + i, ["4:2:0", "4:2:2", "4:4:4"][i % 3],
                                     progressive=bool(i % 2)))
    t = B.ARAwareTransform(512, 16, 0.5, 2.0)
    for i, (data, (st, arr, meta)) in enumerate(zip(datas, ctx.decode_batch(datas))):
        assert st == 0
        w, h = O.jpeg_info(data)[1:3]
        tw, th = t.target_size(w, h)
        ost, dec = O.jpeg_decode(data)
        ref = O.crop_and_resize(dec, tw, th, O.MODE_FIR)
        assert np.array_equal(arr, ref), i


def test_progressive_large_and_restarts():
    L = _lib()
    ctx = L.Context(0)
    ctx.set_option("progressive", 1)
    datas = [_prog(41, 1600, 1100, 92), _prog(42, 1333, 777, 75, "4:4:4", rst=3), _prog(43, 900, 1201, 60, gray=True, rst=5)]
    for data, (st, arr, meta) in zip(datas, ctx.decode_batch(datas)):
        assert st == 0
        ost, ref = O.jpeg_decode(data)
        assert np.array_equal(arr.reshape(ref.shape), ref)


def test_progressive_truncated_is_corrupt():
    L = _lib()
    ctx = L.Context(0)
    ctx.set_option("progressive", 1)
    data = _prog(44, 300, 200)
    res = ctx.decode_batch([data[: len(data) // 2], data])
    assert res[0][0] == L.DG_ERR_CORRUPT and res[1][0] == L.DG_OK


def test_progressive_option_off_is_unsupported():
    L = _lib()
    ctx = L.Context(0)
    ctx.set_option("progressive", 0)
    res = ctx.decode_batch([_prog(45, 64, 48), synth.make_jpeg(46, 64, 48)])
    assert res[0][0] == L.DG_ERR_UNSUPPORTED and res[1][0] == L.DG_OK


def test_progressive_on_by_default():
    """Progressive files decode inline by default (worker_files.rs:14-16 ->
    image -> zune-jpeg decodes them), through the split submission."""
    L = _lib()
    ctx = L.Context(0)
    datas = [_prog(45, 64, 48), synth.make_jpeg(46, 64, 48)]
    for data, (st, arr, _) in zip(datas, ctx.decode_batch(datas)):
        assert st == 0
        ost, ref = O.jpeg_decode(data)
        assert np.array_equal(arr.reshape(ref.shape), ref)
    assert ctx.stat("prog_aggregates") == 1 and ctx.stat("prog_aggregate_images") == 1


def test_progressive_speculative_equals_serial_reader():
    """The speculative-table decoder (scans without restarts) in the
    pipelined single launch against the serial reader launched level by level
    (options prog_serial, prog_pipe) and the oracle, over qualities 1-100
    (long EOB runs at low quality, dense refinements at high quality), all
    samplings and gray, sizes from 1 px to > 64 blocks per chunk row."""
    L = _lib()
    spec_ctx, ser_ctx = L.Context(0), L.Context(0)
    for c in (spec_ctx, ser_ctx):
        c.set_option("progressive", 1)
    ser_ctx.set_option("prog_serial", 1)
    ser_ctx.set_option("prog_pipe", 0)  # serial reader, one launch per level: the round-1 schedule
    datas = []
    for i, q in enumerate([1, 5, 12, 30, 50, 70, 85, 95, 100, 100, 97, 3]):
        rng = np.random.default_rng(900 + i)
        w, h = [(1, 1), (7, 9), (640, 480), (1031, 77), (64, 1500), (333, 333)][i % 6]
        datas.append(_prog(900 + i, w, h, q, ["4:2:0", "4:2:2", "4:4:4"][i % 3], i % 5 == 4))
        datas.append(synth.make_jpeg(950 + i, int(rng.integers(100, 900)), int(rng.integers(100, 900)), q,
                                     progressive=True))
    a, b = spec_ctx.decode_batch(datas), ser_ctx.decode_batch(datas)
    for i, (data, (st, arr, _), (st2, arr2, _)) in enumerate(zip(datas, a, b)):
        assert st == 0 and st2 == 0, (i, L.last_error())
        ost, ref = O.jpeg_decode(data)
        assert np.array_equal(arr.reshape(ref.shape), ref), i
        assert np.array_equal(arr, arr2), i


@pytest.mark.parametrize("lanes", [1, 0])
def test_decode_one_progressive_lane(lanes):
    """dg_decode_one with progressive files among baseline ones: progressive
    callers coalesce into batches of their own (option prog_lanes, default 1)
    that run beside the baseline batches in a slot of their own; every result
    equals the oracle's, and the two kinds never share a batch."""
    import threading
    L = _lib()
    ctx = L.Context(0, crop_and_resize=True, default_image_size=512, downsampling_ratio=16,
                    min_aspect_ratio=0.5, max_aspect_ratio=2.0)
    ctx.set_option("progressive", 1)
    ctx.set_option("prog_lanes", lanes)
    ctx.set_option("coalesce_us", 5000)
    datas = []
    for i in range(48):
        rng = np.random.default_rng(3100 + i)
        datas.append(synth.make_jpeg(3100 + i, int(rng.integers(64, 900)), int(rng.integers(64, 900)),
                                     int(rng.integers(40, 98)), ["4:2:0", "4:2:2", "4:4:4"][i % 3],
                                     progressive=i % 4 == 1))
    res = [None] * len(datas)

    def work(k):
        for i in range(k, len(datas), 12):
            res[i] = ctx.decode_one(datas[i])

    th = [threading.Thread(target=work, args=(k,)) for k in range(12)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    t = B.ARAwareTransform(512, 16, 0.5, 2.0)
    for i, (data, (st, arr, meta)) in enumerate(zip(datas, res)):
        assert st == 0, (i, L.last_error())
        w, h = O.jpeg_info(data)[1:3]
        tw, th_ = t.target_size(w, h)
        ost, dec = O.jpeg_decode(data)
        assert np.array_equal(arr, O.crop_and_resize(dec, tw, th_, O.MODE_FIR)), i
    assert ctx.stat("coalesced_images") == len(datas)


DBG_FORCE_PROG_TIMEOUT = 1 << 19


def test_progressive_wait_timeout_is_unsupported_and_isolated():
    """A scan whose wait for an earlier scan of its image times out stops
    (no reads of blocks a producer may still be writing) and returns its image
    DG_ERR_UNSUPPORTED; baseline images of the same batch stay bit-exact and
    the launch drains.  Test switch: every scan with dependencies times out on
    its first wait."""
    L = _lib()
    ctx = L.Context(0)
    ctx.set_option("progressive", 1)
    ctx.set_option("prog_chain", 0)  # every scan its own wave: chained scans never wait
    prog = [_prog(4701, 300, 200), _prog(4702, 640, 480, 90, "4:4:4")]
    base = [synth.make_jpeg(4703, 320, 240), synth.make_jpeg(4704, 123, 77, 70, "4:2:2")]
    ctx.set_option("debug_flags", DBG_FORCE_PROG_TIMEOUT)
    try:
        res = ctx.decode_batch(prog + base)
    finally:
        ctx.set_option("debug_flags", 0)
    assert [r[0] for r in res[:2]] == [L.DG_ERR_UNSUPPORTED] * 2
    for d, (st, arr, _) in zip(base, res[2:]):
        assert st == 0
        ost, ref = O.jpeg_decode(d)
        assert np.array_equal(arr.reshape(ref.shape), ref)
    assert all(r[0] == 0 for r in ctx.decode_batch(prog))


@pytest.mark.parametrize("chain", [0, 100, 100000])
def test_progressive_chains_bit_exact(chain):
    """Work items of the pipelined launch (option prog_chain): every scan its
    own wave (0), the default (dependency groups chained in one wave unless
    they cost more than the batch's longest scan, so the largest image stays
    pipelined), and every group chained (100000).  The outputs are the
    oracle's in every mode, gray and colour, with and without restarts
    (restart scans use the serial reader inside a chain too)."""
    L = _lib()
    ctx = L.Context(0)
    ctx.set_option("progressive", 1)
    ctx.set_option("prog_chain", chain)
    datas = [_prog(4801, 1700, 1300, 93)] + _cases(48, 14, 420)
    res = ctx.decode_batch(datas)
    for i, (data, (st, arr, _)) in enumerate(zip(datas, res)):
        assert st == 0, (i, L.last_error())
        ost, ref = O.jpeg_decode(data)
        assert np.array_equal(arr.reshape(ref.shape), ref), i
    items, chains = ctx.stat("prog_items"), ctx.stat("prog_chains")
    if chain == 0:
        assert chains == 0
    else:
        assert 0 < chains <= items


def _resized_ref(data, t):
    w, h = O.jpeg_info(data)[1:3]
    tw, th = t.target_size(w, h)
    ost, dec = O.jpeg_decode(data)
    return O.crop_and_resize(dec, tw, th, O.MODE_FIR)


def _mixed(seed, n, every=3):
    out = []
    for i in range(n):
        rng = np.random.default_rng(seed + i)
        out.append(synth.make_jpeg(seed + i, int(rng.integers(64, 700)), int(rng.integers(64, 700)),
                                   int(rng.integers(50, 97)), ["4:2:0", "4:2:2", "4:4:4"][i % 3],
                                   progressive=i % every == 1))
    return out


def test_split_wait_ready_then_wait():
    """dg_submit with progressive members (prog_split, the default): the other
    members form a batch of their own and are complete after dg_wait_ready;
    the progressive ones are pending (meta status DG_ERR_NOT_READY) until
    dg_wait, and then every output equals the oracle's."""
    L = _lib()
    ctx = L.Context(0, crop_and_resize=True, default_image_size=512, downsampling_ratio=16,
                    min_aspect_ratio=0.5, max_aspect_ratio=2.0)
    ctx.set_option("prog_flush_us", 10_000_000)  # launched only by the dg_wait below
    t = B.ARAwareTransform(512, 16, 0.5, 2.0)
    datas = _mixed(8100, 12)
    isp = [i % 3 == 1 for i in range(len(datas))]
    outs = [np.zeros(max(ctx.output_size(d)[1], 1), np.uint8) for d in datas]
    ticket, metas, keep = ctx.submit_host(datas, outs)
    pending = ctx.wait_ready(ticket)
    assert pending == sum(isp)
    for i, d in enumerate(datas):
        if isp[i]:
            assert metas[i].status == L.DG_ERR_NOT_READY, i
        else:
            assert metas[i].status == 0, i
            ref = _resized_ref(d, t)
            assert np.array_equal(outs[i][: ref.size].reshape(ref.shape), ref), i
    ctx.wait(ticket)
    for i, d in enumerate(datas):
        assert metas[i].status == 0, i
        ref = _resized_ref(d, t)
        assert np.array_equal(outs[i][: ref.size].reshape(ref.shape), ref), i
    assert ctx.stat("prog_aggregates") == 1


def test_split_aggregate_launched_before_wait_ready():
    """An aggregate launched while the caller still holds its ticket
    (prog_batch 1: the submission itself launches it) keeps its members'
    metas at DG_ERR_NOT_READY while the GPU decodes -- planning writes the
    batch's own copies, finish() publishes them -- and dg_wait_ready reports
    pending 0 only once outputs and statuses are in place."""
    import time
    L = _lib()
    ctx = L.Context(0, crop_and_resize=True, default_image_size=512, downsampling_ratio=16,
                    min_aspect_ratio=0.5, max_aspect_ratio=2.0)
    ctx.set_option("prog_batch", 1)
    t = B.ARAwareTransform(512, 16, 0.5, 2.0)
    datas = _mixed(8150, 9)
    isp = [i % 3 == 1 for i in range(len(datas))]
    outs = [np.zeros(max(ctx.output_size(d)[1], 1), np.uint8) for d in datas]
    ticket, metas, keep = ctx.submit_host(datas, outs)
    assert ctx.stat("prog_aggregates") >= 1  # launched inside the submission
    for i in range(len(datas)):
        if isp[i]:
            assert metas[i].status == L.DG_ERR_NOT_READY and metas[i].width == 0, i
    deadline = time.time() + 60
    pending = ctx.wait_ready(ticket)
    while pending and time.time() < deadline:
        time.sleep(0.01)
        pending = ctx.wait_ready(ticket)
    assert pending == 0
    for i, d in enumerate(datas):  # complete without dg_wait: outputs copied, metas published
        assert metas[i].status == 0, i
        ref = _resized_ref(d, t)
        assert (metas[i].width, metas[i].height) == (ref.shape[1], ref.shape[0]), i
        assert np.array_equal(outs[i][: ref.size].reshape(ref.shape), ref), i
    ctx.wait(ticket)  # still valid after the members completed


def test_split_aggregates_across_submissions():
    """Progressive members of several submissions share one aggregate batch
    (prog_batch, prog_flush_us large): waited on out of order, every output
    is the oracle's; a later submission starts a new aggregate."""
    L = _lib()
    ctx = L.Context(0)
    ctx.set_option("prog_flush_us", 10_000_000)
    ctx.set_option("prog_batch", 1000)
    subs = [_mixed(8200 + 50 * k, 7, every=2) for k in range(3)]
    held = []
    for datas in subs:
        outs = [np.zeros(max(ctx.output_size(d)[1], 1), np.uint8) for d in datas]
        ticket, metas, keep = ctx.submit_host(datas, outs)
        held.append((ticket, metas, keep, outs, datas))
    for ticket, metas, keep, outs, datas in held:
        assert ctx.wait_ready(ticket) == sum(i % 2 == 1 for i in range(len(datas)))
    for ticket, metas, keep, outs, datas in reversed(held):
        ctx.wait(ticket)
        for i, d in enumerate(datas):
            assert metas[i].status == 0
            ost, ref = O.jpeg_decode(d)
            assert np.array_equal(outs[i][: ref.size].reshape(ref.shape), ref), i
    assert ctx.stat("prog_aggregates") == 1
    assert ctx.stat("prog_aggregate_images") == sum(sum(i % 2 == 1 for i in range(len(d))) for d in subs)
    res = ctx.decode_batch(_mixed(8400, 4, every=2))
    assert all(r[0] == 0 for r in res) and ctx.stat("prog_aggregates") == 2


def test_split_device_path_and_batch_limit():
    """dg_submit_device (coded bytes in HBM, outputs in HBM) splits the same
    way; an aggregate that reaches prog_batch images launches at once."""
    L = _lib()
    ctx = L.Context(0, crop_and_resize=True, default_image_size=512, downsampling_ratio=16,
                    min_aspect_ratio=0.5, max_aspect_ratio=2.0)
    ctx.set_option("prog_batch", 2)
    t = B.ARAwareTransform(512, 16, 0.5, 2.0)
    datas = _mixed(8500, 9)
    res = ctx.decode_batch_torch(datas)
    for i, (d, (st, ten, _)) in enumerate(zip(datas, res)):
        assert st == 0, i
        assert np.array_equal(ten.cpu().numpy(), _resized_ref(d, t)), i
    assert ctx.stat("prog_aggregates") == 1  # launched by the submission that reached prog_batch


def _huff_codes(bits, vals):
    """Canonical Huffman codes (T.81 Annex C) of a DHT (bits[16], vals)."""
    codes, code, k = {}, 0, 0
    for length in range(1, 17):
        for _ in range(bits[length - 1]):
            codes[vals[k]] = (code, length)
            code += 1
            k += 1
        code <<= 1
    return codes


class _Bits:
    def __init__(self):
        self.out, self.acc, self.n = bytearray(), 0, 0

    def put(self, v, n):
        for i in range(n - 1, -1, -1):
            self.acc = (self.acc << 1) | ((v >> i) & 1)
            self.n += 1
            if self.n == 8:
                self.out.append(self.acc)
                if self.acc == 0xFF:
                    self.out.append(0)
                self.acc, self.n = 0, 0

    def done(self):
        if self.n:
            self.put((1 << (8 - self.n)) - 1, 8 - self.n)
        return bytes(self.out)


def _many_scan_jpeg(seed, bw=8, bh=5):
    """A gray progressive JPEG with 65 scans (DC first at Al=1, one AC-first
    scan per zigzag position 1..63, DC refinement): more than the 64 scans a
    deps mask can describe.  Coefficients are drawn directly (quantiser 1),
    Huffman tables are the standard luminance ones (the oracle encoder's)."""
    import ctypes
    from oracle import oracle as O2
    lib = O2.lib()
    dcb = list((ctypes.c_uint8 * 16).in_dll(lib, "oe_dc_luma_bits"))
    dcv = list((ctypes.c_uint8 * 12).in_dll(lib, "oe_dc_vals"))
    acb = list((ctypes.c_uint8 * 16).in_dll(lib, "oe_ac_luma_bits"))
    acv = list((ctypes.c_uint8 * 162).in_dll(lib, "oe_ac_luma_vals"))
    dcc, acc = _huff_codes(dcb, dcv), _huff_codes(acb, acv)
    rng = np.random.default_rng(seed)
    nb = bw * bh
    coef = np.zeros((nb, 64), np.int32)
    coef[:, 0] = rng.integers(-300, 300, nb)
    coef[:, 1:] = rng.integers(-6, 7, (nb, 63)) * (rng.random((nb, 63)) < 0.35)

    def seg(m, body):
        return bytes([0xFF, m]) + (len(body) + 2).to_bytes(2, "big") + body

    def mag(v):
        s = int(abs(v)).bit_length()
        return s, (v if v >= 0 else v + (1 << s) - 1) & ((1 << s) - 1)

    def sos(ss, se, ah, al):
        return seg(0xDA, bytes([1, 1, 0x00, ss, se, (ah << 4) | al]))

    out = bytearray(b"\xFF\xD8")
    out += seg(0xDB, bytes([0]) + bytes([1] * 64))
    out += seg(0xC2, bytes([8]) + (bh * 8).to_bytes(2, "big") + (bw * 8).to_bytes(2, "big") + bytes([1, 1, 0x11, 0]))
    out += seg(0xC4, bytes([0x00]) + bytes(dcb) + bytes(dcv))
    out += seg(0xC4, bytes([0x10]) + bytes(acb) + bytes(acv))
    b, pred = _Bits(), 0
    for i in range(nb):  # DC first, Al = 1
        v = int(coef[i, 0]) >> 1
        s, m = mag(v - pred)
        pred = v
        b.put(*dcc[s])
        b.put(m, s)
    out += sos(0, 0, 0, 1) + b.done()
    for k in range(1, 64):  # one AC-first scan per coefficient
        b = _Bits()
        for i in range(nb):
            v = int(coef[i, k])
            if v == 0:
                b.put(*acc[0x00])  # EOB
            else:
                s, m = mag(v)
                b.put(*acc[s])
                b.put(m, s)
        out += sos(k, k, 0, 0) + b.done()
    b = _Bits()
    for i in range(nb):  # DC refinement: bit 0
        b.put(int(coef[i, 0]) & 1, 1)
    out += sos(0, 0, 1, 0) + b.done() + b"\xFF\xD9"
    return bytes(out)


@pytest.mark.parametrize("chain", [0, 100])
def test_progressive_more_than_64_scans(chain):
    """Files with more scans than a deps mask holds decode, their
    dependency groups always chained; equal to the oracle and to PIL."""
    L = _lib()
    ctx = L.Context(0)
    ctx.set_option("prog_chain", chain)
    datas = [_many_scan_jpeg(9100 + i, 8 + 3 * i, 5 + i) for i in range(3)] + [_prog(9200, 300, 200)]
    for data, (st, arr, _) in zip(datas, ctx.decode_batch(datas)):
        assert st == 0, L.last_error()
        ost, ref = O.jpeg_decode(data)
        assert ost == 0
        pil = np.asarray(Image.open(io.BytesIO(data)))
        assert np.array_equal(ref.reshape(pil.shape), pil)
        assert np.array_equal(arr.reshape(ref.shape), ref)
