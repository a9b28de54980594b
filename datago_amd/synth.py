"""Seeded synthetic JPEG corpora for tests and bench.py.

Content = smooth gradients + random rectangles/ellipses + N(0, 8) noise, encoded
by PIL/libjpeg-turbo (baseline, standard tables, optionally restart markers).
There is no dataset on the box (no network), so every corpus is generated from
a seed.  This module is bench/test plumbing, not part of the decode path.
"""
from __future__ import annotations

import io
import math
from typing import List, Optional, Tuple

import numpy as np
from PIL import Image, ImageDraw

SUBSAMPLING = {"4:4:4": 0, "4:2:2": 1, "4:2:0": 2}


def synth_pixels(rng: np.random.Generator, w: int, h: int, gray: bool = False) -> np.ndarray:
    """Smooth gradient + a few shapes + gaussian noise, uint8 HWC (or HW).

    Worked in 64-row bands so the float temporaries stay in cache; every
    element sees the same operations in the same order and the RNG is drawn
    in the same sequence, so the pixels equal the whole-image formulation."""
    c = 1 if gray else 3
    # low-resolution random field upsampled bilinearly -> smooth gradients
    gh, gw = max(2, h // 64 + 2), max(2, w // 64 + 2)
    grid = rng.uniform(0, 255, size=(gh, gw, c)).astype(np.float32)
    ys = np.linspace(0, gh - 1, h, dtype=np.float32)
    xs = np.linspace(0, gw - 1, w, dtype=np.float32)
    y0 = np.floor(ys).astype(np.int32).clip(0, gh - 2)
    x0 = np.floor(xs).astype(np.int32).clip(0, gw - 2)
    fys = ys - y0
    fx = (xs - x0)[None, :, None]
    g0, g1 = grid[:, x0], grid[:, x0 + 1]
    base = np.empty((h, w, c), np.uint8)
    R = 64
    for r0 in range(0, h, R):
        r1 = min(h, r0 + R)
        fy = fys[r0:r1, None, None]
        yy = y0[r0:r1]
        a, b, cc, d = g0[yy], g1[yy], g0[yy + 1], g1[yy + 1]
        img = (a * (1 - fx) * (1 - fy) + b * fx * (1 - fy) + cc * (1 - fx) * fy + d * fx * fy)
        base[r0:r1] = img.clip(0, 255).astype(np.uint8)
    im = Image.fromarray(base[:, :, 0] if gray else base)
    dr = ImageDraw.Draw(im)
    for _ in range(int(rng.integers(2, 8))):
        x1, x2 = sorted(rng.integers(0, w, 2).tolist())
        y1, y2 = sorted(rng.integers(0, h, 2).tolist())
        col = int(rng.integers(0, 256)) if gray else tuple(int(v) for v in rng.integers(0, 256, 3))
        if rng.random() < 0.5:
            dr.rectangle([x1, y1, x2, y2], fill=col)
        else:
            dr.ellipse([x1, y1, x2, y2], fill=col)
    arr = np.asarray(im)
    out = np.empty(arr.shape, np.uint8)
    for r0 in range(0, h, R):  # N(0, 8) noise, drawn band by band in stream order
        r1 = min(h, r0 + R)
        blk = arr[r0:r1].astype(np.int16)
        out[r0:r1] = (blk + rng.normal(0, 8, size=blk.shape)).clip(0, 255).astype(np.uint8)
    return out


def encode_jpeg(arr: np.ndarray, quality: int = 90, subsampling: str = "4:2:0",
                restart_marker_rows: int = 0, restart_marker_blocks: int = 0, progressive: bool = False) -> bytes:
    im = Image.fromarray(arr)
    buf = io.BytesIO()
    kw = dict(quality=int(quality), progressive=bool(progressive))
    if im.mode == "RGB":
        kw["subsampling"] = SUBSAMPLING[subsampling]
    if restart_marker_rows:
        kw["restart_marker_rows"] = int(restart_marker_rows)
    if restart_marker_blocks:
        kw["restart_marker_blocks"] = int(restart_marker_blocks)
    im.save(buf, format="JPEG", **kw)
    return buf.getvalue()


def make_jpeg(seed: int, w: int, h: int, quality: int = 90, subsampling: str = "4:2:0",
              gray: bool = False, restart_marker_rows: int = 0, progressive: bool = False) -> bytes:
    rng = np.random.default_rng(seed)
    return encode_jpeg(synth_pixels(rng, w, h, gray), quality, subsampling, restart_marker_rows,
                       progressive=progressive)


def make_cmyk_jpeg(seed: int, w: int, h: int, quality: int = 90) -> bytes:
    """A 4-component (Adobe CMYK) JPEG: valid, outside the GPU path."""
    rng = np.random.default_rng(seed)
    buf = io.BytesIO()
    Image.fromarray(synth_pixels(rng, w, h)).convert("CMYK").save(buf, format="JPEG", quality=int(quality))
    return buf.getvalue()


def mixed_spec(seed: int, n: int, short_min: int = 256, short_max: int = 2048,
               ar_min: float = 0.4, ar_max: float = 2.5) -> List[Tuple[int, int, int, str, bool]]:
    """BASELINE configs[1] distribution: AR log-uniform [0.4,2.5], short side
    U[short_min, short_max], q U{75..95}, 80% 4:2:0 / 10% 4:2:2 / 10% 4:4:4,
    5% grayscale."""
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        ar = math.exp(rng.uniform(math.log(ar_min), math.log(ar_max)))
        short = int(rng.integers(short_min, short_max + 1))
        if ar >= 1.0:
            w, h = int(round(short * ar)), short
        else:
            w, h = short, int(round(short / ar))
        q = int(rng.integers(75, 96))
        u = rng.random()
        ss = "4:2:0" if u < 0.8 else ("4:2:2" if u < 0.9 else "4:4:4")
        gray = bool(rng.random() < 0.05)
        out.append((w, h, q, ss, gray))
    return out


def _make_one(args):
    seed, (w, h, q, ss, gray), rst = args[:3]
    prog = args[3] if len(args) > 3 else False
    return make_jpeg(seed, w, h, q, ss, gray, rst, progressive=prog)


def _pool_map(jobs, workers):
    # close + join (not the context manager's terminate): workers that get
    # SIGTERM under a profiler's signal handler can hang the parent's join
    import multiprocessing as mp
    pool = mp.get_context("fork").Pool(workers)
    try:
        out = pool.map(_make_one, jobs, chunksize=4)
    finally:
        pool.close()
        pool.join()
    return out


def mixed_corpus(seed: int, n: int, short_min: int = 256, short_max: int = 2048,
                 workers: int = 1, restart_marker_rows: int = 0, lo: int = 0, hi: int | None = None,
                 progressive_frac: float = 0.0) -> List[bytes]:
    """Images [lo, hi) of the logical n-image stream for `seed` (a rank's
    slice of a sharded corpus is generated without building the rest).
    progressive_frac: share of images written as progressive JPEGs (libjpeg's
    default script), every 1/frac-th image of the stream."""
    spec = mixed_spec(seed, n, short_min, short_max)
    hi = n if hi is None else hi
    step = int(round(1.0 / progressive_frac)) if progressive_frac > 0 else 0
    jobs = [(seed * 1_000_003 + i, spec[i], restart_marker_rows, bool(step) and i % step == 0) for i in range(lo, hi)]
    if workers > 1:
        return _pool_map(jobs, workers)
    return [_make_one(j) for j in jobs]


def corpus_cache_dir() -> str:
    """Where generated pool images are kept between runs on one machine
    ($DATAGO_CORPUS_CACHE, default <tmp>/datago_amd_corpus): the bench's
    back-to-back 1/2/4/8-GPU runs, and the ranks of one run, share it."""
    import os
    import tempfile
    return os.environ.get("DATAGO_CORPUS_CACHE") or os.path.join(tempfile.gettempdir(), "datago_amd_corpus")


def is_progressive_jpeg(data: bytes) -> bool:
    """SOF2 before the first SOS (what the library's sniff checks)."""
    i, n = 2, len(data)
    if n < 4 or data[0] != 0xFF or data[1] != 0xD8:
        return False
    while i + 4 <= n:
        if data[i] != 0xFF:
            return False
        m = data[i + 1]
        if m == 0xFF:
            i += 1
            continue
        if m == 0xC2:
            return True
        if m in (0xC0, 0xC1, 0xDA) or m == 0xD9:
            return False
        if 0xD0 <= m <= 0xD7 or m == 0x01:
            i += 2
            continue
        i += 2 + ((data[i + 2] << 8) | data[i + 3])
    return False


def _pool_job(seed: int, i: int, spec, progressive_frac: float, restart_marker_rows: int = 0):
    step = int(round(1.0 / progressive_frac)) if progressive_frac > 0 else 0
    return (seed * 1_000_003 + i, spec[i], int(restart_marker_rows), bool(step) and i % step == 0)


def _cache_name(job) -> str:
    s, (w, h, q, ss, gray), rst, prog = job
    return f"v1_{s}_{w}x{h}_q{q}_{ss.replace(':', '')}_{int(gray)}_{rst}_{int(prog)}.jpg"


def _make_cached(args):
    import os
    job, path = args
    data = _make_one(job)
    tmp = f"{path}.{os.getpid()}.tmp"
    with open(tmp, "wb") as f:
        f.write(data)
    os.replace(tmp, path)  # atomic: concurrent ranks never see a partial file
    return len(data)


def generate_pool_images(seed: int, n_pool: int, indices, workers: int = 1, short_min: int = 256,
                         short_max: int = 2048, progressive_frac: float = 0.0, cache_dir: str | None = None,
                         progress=None, restart_marker_rows: int = 0) -> int:
    """Make sure pool images `indices` of the seed's n_pool-image pool (the
    mixed_spec distribution; image i is exactly mixed_corpus(seed, n_pool)[i])
    exist in the cache.  Returns how many were generated."""
    import os
    import time
    cache_dir = cache_dir or corpus_cache_dir()
    os.makedirs(cache_dir, exist_ok=True)
    spec = mixed_spec(seed, n_pool, short_min, short_max)
    todo = []
    for i in indices:
        job = _pool_job(seed, i, spec, progressive_frac, restart_marker_rows)
        path = os.path.join(cache_dir, _cache_name(job))
        if not os.path.exists(path):
            todo.append((job, path))
    if not todo:
        return 0
    t0, last = time.time(), time.time()
    if workers > 1:
        import multiprocessing as mp
        pool = mp.get_context("fork").Pool(workers)
        try:
            for k, _ in enumerate(pool.imap_unordered(_make_cached, todo, chunksize=2)):
                if progress and time.time() - last > 20:
                    last = time.time()
                    progress(f"corpus: {k + 1}/{len(todo)} images generated in {last - t0:.0f} s")
        finally:
            pool.close()
            pool.join()
    else:
        for t in todo:
            _make_cached(t)
    return len(todo)


def load_pool_images(seed: int, n_pool: int, indices, short_min: int = 256, short_max: int = 2048,
                     progressive_frac: float = 0.0, cache_dir: str | None = None,
                     restart_marker_rows: int = 0) -> List[bytes]:
    import os
    cache_dir = cache_dir or corpus_cache_dir()
    spec = mixed_spec(seed, n_pool, short_min, short_max)
    out = []
    for i in indices:
        with open(os.path.join(cache_dir, _cache_name(_pool_job(seed, i, spec, progressive_frac,
                                                               restart_marker_rows))), "rb") as f:
            out.append(f.read())
    return out


def uniform_corpus(seed: int, n: int, w: int = 640, h: int = 480, quality: int = 90,
                   subsampling: str = "4:2:0", workers: int = 1) -> List[bytes]:
    jobs = [(seed * 1_000_003 + i, (w, h, quality, subsampling, False), 0) for i in range(n)]
    if workers > 1:
        return _pool_map(jobs, workers)
    return [_make_one(j) for j in jobs]


# ------------------------------------------------- JPEG with chosen Huffman tables
#
# PIL always writes libjpeg's Annex K Huffman tables unless optimize=True, and
# even its optimised tables stay shallow on synthetic content.  Real corpora
# (mozjpeg, per-image optimised web JPEGs) carry tables with long (10..16-bit)
# codes spread over many 9-bit prefixes -- the decoder's second-level and
# fallback lookups.  This small baseline encoder (T.81 sequential Huffman,
# 8-bit, gray / 4:4:4 / 4:2:0, optional restart interval) writes the same
# coefficients with either optimal length-limited tables (Annex K.2/K.3, as
# optimize=True) or deliberately deep ones.  Test data only: the decoded
# pixels are checked against the oracle and PIL, never against this encoder.

_STD_LUMA_Q = [16, 11, 10, 16, 24, 40, 51, 61, 12, 12, 14, 19, 26, 58, 60, 55, 14, 13, 16, 24, 40, 57, 69, 56,
               14, 17, 22, 29, 51, 87, 80, 62, 18, 22, 37, 56, 68, 109, 103, 77, 24, 35, 55, 64, 81, 104, 113, 92,
               49, 64, 78, 87, 103, 121, 120, 101, 72, 92, 95, 98, 112, 100, 103, 99]
_STD_CHROMA_Q = [17, 18, 24, 47, 99, 99, 99, 99, 18, 21, 26, 66, 99, 99, 99, 99, 24, 26, 56, 99, 99, 99, 99, 99,
                 47, 66, 99, 99, 99, 99, 99, 99] + [99] * 32
_ZIGZAG = [0, 1, 8, 16, 9, 2, 3, 10, 17, 24, 32, 25, 18, 11, 4, 5, 12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6, 7,
           14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39,
           46, 53, 60, 61, 54, 47, 55, 62, 63]


def _scaled_q(base, quality):
    scale = 5000 // quality if quality < 50 else 200 - 2 * quality
    return [min(255, max(1, (b * scale + 50) // 100)) for b in base]


def _huff_optimal(freq):
    """Annex K.2 code sizes + K.3 16-bit limit: (bits[1..16], vals)."""
    freq = list(freq) + [1]  # reserved symbol 256: no code of all ones
    n = len(freq)
    size = [0] * n
    others = [-1] * n
    f = [x if x > 0 else 0 for x in freq]
    while True:
        c1 = c2 = -1
        for i in range(n):  # least frequency, highest index on ties (libjpeg jchuff)
            if f[i] and (c1 < 0 or f[i] <= f[c1]):
                c1 = i
        for i in range(n):
            if f[i] and i != c1 and (c2 < 0 or f[i] <= f[c2]):
                c2 = i
        if c2 < 0:
            break
        f[c1] += f[c2]
        f[c2] = 0
        size[c1] += 1
        while others[c1] >= 0:
            c1 = others[c1]
            size[c1] += 1
        others[c1] = c2
        size[c2] += 1
        while others[c2] >= 0:
            c2 = others[c2]
            size[c2] += 1
    bits = [0] * 33
    for i in range(n):
        if size[i]:
            bits[size[i]] += 1
    for i in range(32, 16, -1):
        while bits[i] > 0:
            j = i - 2
            while bits[j] == 0:
                j -= 1
            bits[i] -= 2
            bits[i - 1] += 1
            bits[j + 1] += 2
            bits[j] -= 1
    i = 16
    while bits[i] == 0:
        i -= 1
    bits[i] -= 1  # drop the reserved code
    vals = [s for L in range(1, 33) for s in range(n - 1) if size[s] == L]
    return [0] + bits[1:17], vals


def _huff_deep(freq, short, mid_len, mid_n):
    """Deliberately deep table over every symbol with nonzero frequency (and
    the rest of `universe`): the `short` most frequent get 1..short-bit codes,
    the next mid_n get mid_len-bit codes, the rest 16-bit codes."""
    order = sorted(range(len(freq)), key=lambda s: (-freq[s], s))
    order = [s for s in order if freq[s] > 0] + [s for s in order if freq[s] == 0]
    bits = [0] * 17
    vals = []
    for k, sym in enumerate(order):
        L = (k + 1) if k < short else (mid_len if k < short + mid_n else 16)
        bits[L] += 1
        vals.append(sym)
    by_len = sorted(zip([((k + 1) if k < short else (mid_len if k < short + mid_n else 16))
                         for k in range(len(order))], range(len(order))))
    return bits, [order[i] for _, i in by_len]


def _huff_codes(bits, vals):
    codes, code, k = {}, 0, 0
    for L in range(1, 17):
        for _ in range(bits[L]):
            codes[vals[k]] = (code, L)
            code += 1
            k += 1
        code <<= 1
    return codes


class _BitWriter:
    def __init__(self):
        self.out = bytearray()
        self.acc = 0
        self.n = 0

    def put(self, v, n):
        self.acc = (self.acc << n) | (v & ((1 << n) - 1))
        self.n += n
        while self.n >= 8:
            b = (self.acc >> (self.n - 8)) & 0xFF
            self.out.append(b)
            if b == 0xFF:
                self.out.append(0)
            self.n -= 8
        self.acc &= (1 << self.n) - 1

    def pad(self):
        if self.n:
            self.put((1 << (8 - self.n)) - 1, 8 - self.n)


def _category(v):
    return 0 if v == 0 else int(abs(v)).bit_length()


def encode_jpeg_tables(arr: np.ndarray, quality: int = 75, subsampling: str = "4:2:0", tables: str = "optimal",
                       restart_interval: int = 0) -> bytes:
    """Baseline JPEG of `arr` (HW gray or HWC RGB) with Huffman tables
    `tables` = "optimal" (per-image, as optimize=True / mozjpeg) or "deep"
    (10- and 16-bit codes over many 9-bit prefixes: the decoder's sub-table
    overflow path)."""
    arr = np.asarray(arr)
    gray = arr.ndim == 2
    h, w = arr.shape[:2]
    if gray:
        planes = [arr.astype(np.float64)]
        samp = [(1, 1)]
    else:
        r, g, b = [arr[:, :, i].astype(np.float64) for i in range(3)]
        planes = [0.299 * r + 0.587 * g + 0.114 * b,
                  -0.168735892 * r - 0.331264108 * g + 0.5 * b + 128,
                  0.5 * r - 0.418687589 * g - 0.081312411 * b + 128]
        samp = [(2, 2), (1, 1), (1, 1)] if subsampling == "4:2:0" else [(1, 1)] * 3
    hmax, vmax = max(s[0] for s in samp), max(s[1] for s in samp)
    mx, my = -(-w // (8 * hmax)), -(-h // (8 * vmax))
    qt = [_scaled_q(_STD_LUMA_Q, quality), _scaled_q(_STD_CHROMA_Q, quality)]
    k = np.arange(8)
    C = np.sqrt(2 / 8) * np.cos((2 * k[None, :] + 1) * k[:, None] * np.pi / 16)
    C[0, :] = np.sqrt(1 / 8)
    comps = []
    for ci, (p, (hs, vs)) in enumerate(zip(planes, samp)):
        if (hs, vs) != (hmax, vmax):  # 2x2 box average, edge replicated
            pp = np.pad(p, ((0, h % 2), (0, w % 2)), mode="edge")
            p = (pp[0::2, 0::2] + pp[1::2, 0::2] + pp[0::2, 1::2] + pp[1::2, 1::2]) / 4
        bw, bh = mx * hs, my * vs
        p = np.pad(p, ((0, bh * 8 - p.shape[0]), (0, bw * 8 - p.shape[1])), mode="edge") - 128.0
        blk = p.reshape(bh, 8, bw, 8).transpose(0, 2, 1, 3)
        d = np.einsum("ij,abjk,lk->abil", C, blk, C)
        q = np.array(qt[0 if ci == 0 else 1], np.float64).reshape(8, 8)
        zz = np.rint(d / q).astype(np.int64).reshape(bh, bw, 64)[:, :, _ZIGZAG]
        comps.append(zz)
    # symbol streams: MCU order, per component (DC diff, AC run/size), RST resets
    seq = []  # (component, kind 0=dc 1=ac, symbol, extra value, extra bits) or ("rst", n)
    pred = [0] * len(comps)
    nmcu = 0
    for my_ in range(my):
        for mx_ in range(mx):
            if restart_interval and nmcu and nmcu % restart_interval == 0:
                seq.append(("rst", (nmcu // restart_interval - 1) & 7))
                pred = [0] * len(comps)
            nmcu += 1
            for ci, (hs, vs) in enumerate(samp):
                for by in range(vs):
                    for bx in range(hs):
                        z = comps[ci][my_ * vs + by, mx_ * hs + bx]
                        diff = int(z[0]) - pred[ci]
                        pred[ci] = int(z[0])
                        s_ = _category(diff)
                        seq.append((ci, 0, s_, diff, s_))
                        run = 0
                        last = 63
                        while last > 0 and z[last] == 0:
                            last -= 1
                        for kk in range(1, last + 1):
                            v = int(z[kk])
                            if v == 0:
                                run += 1
                                continue
                            while run > 15:
                                seq.append((ci, 1, 0xF0, 0, 0))
                                run -= 16
                            s_ = _category(v)
                            seq.append((ci, 1, (run << 4) | s_, v, s_))
                            run = 0
                        if last < 63:
                            seq.append((ci, 1, 0x00, 0, 0))
    # tables: 0 = luma, 1 = chroma
    freqs = [[[0] * 256 for _ in range(2)] for _ in range(2)]  # [kind][table][symbol]
    for e in seq:
        if e[0] != "rst":
            freqs[e[1]][0 if e[0] == 0 else 1][e[2]] += 1
    specs = [[None, None], [None, None]]
    for kind in range(2):
        for t in range(1 if gray else 2):
            f = freqs[kind][t]
            if tables == "deep":
                if kind == 0:
                    f = [f[s] if s < 12 else 0 for s in range(12)]
                    specs[kind][t] = _huff_deep([x + 1 for x in f], 1, 12, 5)
                else:
                    uni = [0x00, 0xF0] + [(r_ << 4) | s_ for r_ in range(16) for s_ in range(1, 11)]
                    ff = [f[s] for s in uni]
                    bits, vi = _huff_deep(ff, 1, 10, 100)
                    specs[kind][t] = (bits, [uni[i] for i in vi])
            else:
                if kind == 0:
                    f = f[:12]
                bits, vals = _huff_optimal(f)
                specs[kind][t] = (bits, vals)
    codes = [[_huff_codes(*specs[kind][t]) if specs[kind][t] else None for t in range(2)] for kind in range(2)]
    bw_ = _BitWriter()
    for e in seq:
        if e[0] == "rst":
            bw_.pad()
            bw_.out += bytes([0xFF, 0xD0 + e[1]])
            continue
        ci, kind, sym, v, nb = e
        code, L = codes[kind][0 if ci == 0 else 1][sym]
        bw_.put(code, L)
        if nb:
            bw_.put(v if v >= 0 else v + (1 << nb) - 1, nb)
    bw_.pad()
    # markers
    out = bytearray(b"\xff\xd8")
    out += b"\xff\xe0\x00\x10JFIF\x00\x01\x01\x00\x00\x01\x00\x01\x00\x00"
    for t in range(1 if gray else 2):
        out += b"\xff\xdb\x00\x43" + bytes([t]) + bytes(qt[t][z] for z in _ZIGZAG)  # zigzag order
    nc = len(comps)
    out += b"\xff\xc0" + (8 + 3 * nc).to_bytes(2, "big") + b"\x08" + h.to_bytes(2, "big") + w.to_bytes(2, "big") \
        + bytes([nc])
    for ci, (hs, vs) in enumerate(samp):
        out += bytes([ci + 1, (hs << 4) | vs, 0 if ci == 0 else 1])
    for kind in range(2):
        for t in range(1 if gray else 2):
            bits, vals = specs[kind][t]
            body = bytes([(kind << 4) | t]) + bytes(bits[1:17]) + bytes(vals)
            out += b"\xff\xc4" + (len(body) + 2).to_bytes(2, "big") + body
    if restart_interval:
        out += b"\xff\xdd\x00\x04" + int(restart_interval).to_bytes(2, "big")
    out += b"\xff\xda" + (6 + 2 * nc).to_bytes(2, "big") + bytes([nc])
    for ci in range(nc):
        out += bytes([ci + 1, 0x00 if ci == 0 else 0x11])
    out += b"\x00\x3f\x00"
    out += bw_.out + b"\xff\xd9"
    return bytes(out)


# ---------------------------------------------------------------- PNG

PNG_KINDS = ("L", "LA", "RGB", "RGBA", "P8", "P8T", "P4", "P2", "P1", "L1", "L2", "L4", "LT", "RGBT")


def _png_chunk(t: bytes, data: bytes) -> bytes:
    import struct
    import zlib
    return struct.pack(">I", len(data)) + t + data + struct.pack(">I", zlib.crc32(t + data) & 0xFFFFFFFF)


def _paeth(a, b, c):
    p = a + b - c
    pa, pb, pc = np.abs(p - a), np.abs(p - b), np.abs(p - c)
    return np.where((pa <= pb) & (pa <= pc), a, np.where(pb <= pc, b, c))


def png_filter_rows(rows: np.ndarray, bpp: int, filters: np.ndarray) -> bytes:
    """PNG scanline filtering (spec 9.2) of H x rowbytes uint8 with the given
    per-row filter types; returns the filtered stream (filter byte + row)."""
    h, rb = rows.shape
    out = bytearray()
    prev = np.zeros(rb, np.int32)
    for y in range(h):
        r = rows[y].astype(np.int32)
        a = np.concatenate([np.zeros(bpp, np.int32), r[:-bpp]]) if rb > bpp else np.zeros(rb, np.int32)
        c = np.concatenate([np.zeros(bpp, np.int32), prev[:-bpp]]) if rb > bpp else np.zeros(rb, np.int32)
        f = int(filters[y])
        if f == 0:
            v = r
        elif f == 1:
            v = r - a
        elif f == 2:
            v = r - prev
        elif f == 3:
            v = r - ((a + prev) >> 1)
        else:
            v = r - _paeth(a, prev, c)
        out.append(f)
        out += (v & 0xFF).astype(np.uint8).tobytes()
        prev = r
    return bytes(out)


ADAM7 = ((0, 0, 8, 8), (4, 0, 8, 8), (0, 4, 4, 8), (2, 0, 4, 4), (0, 2, 2, 4), (1, 0, 2, 2), (0, 1, 1, 2))


def _filters(n: int, filters: str, rng: np.random.Generator) -> np.ndarray:
    if filters == "random":
        return rng.integers(0, 5, size=n)
    if filters == "none":
        return np.zeros(n, np.int64)
    return np.full(n, int(filters))


def encode_png(rows: np.ndarray, w: int, h: int, depth: int, ctype: int, bpp: int, rng: np.random.Generator,
               level: int = 6, strategy: int = 0, filters: str = "random", idat_max: int = 0,
               plte: Optional[bytes] = None, trns: Optional[bytes] = None, samples: Optional[np.ndarray] = None,
               interlace: bool = False) -> bytes:
    """PNG writer for test corpora: explicit filter choice ("random" per row,
    "none", or a filter number), zlib level/strategy (0 = stored blocks,
    Z_FIXED = fixed Huffman), IDAT split into chunks of at most idat_max.
    interlace: Adam7 (PNG spec 8.2) from `samples` (h, w, spp) -- 8-bit
    samples, or sample values for depths 1/2/4 -- each pass filtered on its own."""
    import struct
    import zlib
    if interlace:
        parts = []
        for x0, y0, dx, dy in ADAM7:
            sub = samples[y0::dy, x0::dx]
            if sub.shape[0] == 0 or sub.shape[1] == 0:
                continue
            if depth < 8:
                prow = _pack_bits(sub[:, :, 0], depth)
            else:
                prow = sub.reshape(sub.shape[0], -1)
            parts.append(png_filter_rows(prow, bpp, _filters(sub.shape[0], filters, rng)))
        raw = b"".join(parts)
    else:
        raw = png_filter_rows(rows, bpp, _filters(h, filters, rng))
    co = zlib.compressobj(level, zlib.DEFLATED, 15, 8, strategy)
    z = co.compress(raw) + co.flush()
    out = b"\x89PNG\r\n\x1a\n" + _png_chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, depth, ctype, 0, 0,
                                                                     1 if interlace else 0))
    if plte is not None:
        out += _png_chunk(b"PLTE", plte)
    if trns is not None:
        out += _png_chunk(b"tRNS", trns)
    step = idat_max if idat_max > 0 else len(z)
    for i in range(0, max(len(z), 1), max(step, 1)):
        out += _png_chunk(b"IDAT", z[i:i + step])
    return out + _png_chunk(b"IEND", b"")


def _pack_bits(idx: np.ndarray, depth: int) -> np.ndarray:
    h, w = idx.shape
    per = 8 // depth
    rb = (w * depth + 7) // 8
    pad = np.zeros((h, rb * per), np.uint8)
    pad[:, :w] = idx
    pad = pad.reshape(h, rb, per)
    out = np.zeros((h, rb), np.uint8)
    for k in range(per):
        out |= (pad[:, :, k] << (8 - depth * (k + 1))).astype(np.uint8)
    return out


def make_png(seed: int, w: int, h: int, kind: str = "RGB", **kw) -> bytes:
    """Seeded PNG of the given kind (PNG_KINDS).  Pixel content as synth_pixels;
    alpha is a smooth ramp with fully transparent/opaque patches."""
    rng = np.random.default_rng(seed)
    gray = kind[0] == "L" or kind[0] == "P"
    px = synth_pixels(rng, w, h, gray=gray)
    px = px.reshape(h, w, -1)
    alpha = np.clip(np.linspace(-64, 320, w)[None, :] + rng.normal(0, 30, (h, w)), 0, 255).astype(np.uint8)
    plte = trns = None
    if kind in ("L", "LA", "RGB", "RGBA"):
        if kind in ("LA", "RGBA"):
            px = np.concatenate([px, alpha[:, :, None]], axis=2)
        depth, ctype = 8, {"L": 0, "LA": 4, "RGB": 2, "RGBA": 6}[kind]
        c = px.shape[2]
        rows = px.reshape(h, w * c)
        samples = px
        bpp = c
    elif kind.startswith("P"):
        depth = int(kind[1])
        ncol = 1 << depth
        npal = int(rng.integers(max(1, ncol // 2), ncol + 1))
        pal = rng.integers(0, 256, size=(npal, 3)).astype(np.uint8)
        idx = (px[:, :, 0].astype(np.int32) * ncol // 256).astype(np.uint8)  # may exceed npal: black
        plte = pal.tobytes()
        if kind.endswith("T"):
            trns = rng.integers(0, 256, size=int(rng.integers(1, npal + 1))).astype(np.uint8).tobytes()
        ctype = 3
        rows = idx if depth == 8 else _pack_bits(idx, depth)
        samples = idx[:, :, None]
        bpp = 1
    elif kind in ("L1", "L2", "L4"):
        depth = int(kind[1])
        v = (px[:, :, 0].astype(np.int32) >> (8 - depth)).astype(np.uint8)
        ctype, bpp = 0, 1
        rows = _pack_bits(v, depth)
        samples = v[:, :, None]
        if kw.pop("trns_key", False):
            trns = bytes([0, int(v[0, 0])])
    elif kind == "LT":
        depth, ctype, bpp = 8, 0, 1
        rows = px[:, :, 0].copy()
        samples = rows[:, :, None]
        trns = bytes([0, int(rows[0, 0])])
    elif kind == "RGBT":
        depth, ctype, bpp = 8, 2, 3
        rows = px.reshape(h, w * 3)
        samples = px
        trns = bytes([0, int(px[0, 0, 0]), 0, int(px[0, 0, 1]), 0, int(px[0, 0, 2])])
    else:
        raise ValueError(kind)
    return encode_png(rows, w, h, depth, ctype, bpp, rng, plte=plte, trns=trns, samples=samples, **kw)


def pil_png(arr: np.ndarray, **kw) -> bytes:
    """PNG through PIL's own encoder (what most PNGs in the wild look like)."""
    im = Image.fromarray(arr)
    buf = io.BytesIO()
    im.save(buf, format="PNG", **kw)
    return buf.getvalue()


# ---------------------------------------------------------------- WebDataset shards

def imagenet_like_spec(seed: int, n: int):
    """BASELINE configs[2]: fake-imagenet-like members, W U[300,500], H U[250,500], q90."""
    rng = np.random.default_rng(seed)
    return [(int(rng.integers(300, 501)), int(rng.integers(250, 501)), int(rng.integers(0, 1000))) for _ in range(n)]


def _wds_member(args):
    seed, (w, h, cls) = args
    return make_jpeg(seed, w, h, 90, "4:2:0"), str(cls).encode()


def make_wds_shard(seed: int, n: int, first_key: int = 0, workers: int = 1, fmt: str = "gnu") -> bytes:
    """A WebDataset tar: {key}.jpg + {key}.cls per sample (tarfile, GNU format)."""
    import tarfile
    spec = imagenet_like_spec(seed, n)
    jobs = [(seed * 1_000_003 + i, spec[i]) for i in range(n)]
    if workers > 1:
        import multiprocessing as mp
        p = mp.get_context("fork").Pool(workers)
        try:
            members = p.map(_wds_member, jobs, chunksize=4)
        finally:
            p.close()
            p.join()
    else:
        members = [_wds_member(j) for j in jobs]
    buf = io.BytesIO()
    tf_fmt = {"gnu": tarfile.GNU_FORMAT, "pax": tarfile.PAX_FORMAT, "ustar": tarfile.USTAR_FORMAT}[fmt]
    with tarfile.open(fileobj=buf, mode="w", format=tf_fmt) as tf:
        for i, (jpg, cls) in enumerate(members):
            key = f"n{first_key + i:08d}"
            for name, data in ((f"{key}.jpg", jpg), (f"{key}.cls", cls)):
                ti = tarfile.TarInfo(name)
                ti.size = len(data)
                ti.mtime = 0
                tf.addfile(ti, io.BytesIO(data))
    return buf.getvalue()
