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
    """Smooth gradient + a few shapes + gaussian noise, uint8 HWC (or HW)."""
    c = 1 if gray else 3
    # low-resolution random field upsampled bilinearly -> smooth gradients
    gh, gw = max(2, h // 64 + 2), max(2, w // 64 + 2)
    grid = rng.uniform(0, 255, size=(gh, gw, c)).astype(np.float32)
    ys = np.linspace(0, gh - 1, h, dtype=np.float32)
    xs = np.linspace(0, gw - 1, w, dtype=np.float32)
    y0 = np.floor(ys).astype(np.int32).clip(0, gh - 2)
    x0 = np.floor(xs).astype(np.int32).clip(0, gw - 2)
    fy = (ys - y0)[:, None, None]
    fx = (xs - x0)[None, :, None]
    a = grid[y0][:, x0]
    b = grid[y0][:, x0 + 1]
    cc = grid[y0 + 1][:, x0]
    d = grid[y0 + 1][:, x0 + 1]
    img = (a * (1 - fx) * (1 - fy) + b * fx * (1 - fy) + cc * (1 - fx) * fy + d * fx * fy)
    im = Image.fromarray(img.clip(0, 255).astype(np.uint8)[:, :, 0] if gray else
                         img.clip(0, 255).astype(np.uint8))
    dr = ImageDraw.Draw(im)
    for _ in range(int(rng.integers(2, 8))):
        x1, x2 = sorted(rng.integers(0, w, 2).tolist())
        y1, y2 = sorted(rng.integers(0, h, 2).tolist())
        col = int(rng.integers(0, 256)) if gray else tuple(int(v) for v in rng.integers(0, 256, 3))
        if rng.random() < 0.5:
            dr.rectangle([x1, y1, x2, y2], fill=col)
        else:
            dr.ellipse([x1, y1, x2, y2], fill=col)
    arr = np.asarray(im).astype(np.int16)
    noise = rng.normal(0, 8, size=arr.shape)
    return (arr + noise).clip(0, 255).astype(np.uint8)


def encode_jpeg(arr: np.ndarray, quality: int = 90, subsampling: str = "4:2:0",
                restart_marker_rows: int = 0, restart_marker_blocks: int = 0) -> bytes:
    im = Image.fromarray(arr)
    buf = io.BytesIO()
    kw = dict(quality=int(quality))
    if im.mode == "RGB":
        kw["subsampling"] = SUBSAMPLING[subsampling]
    if restart_marker_rows:
        kw["restart_marker_rows"] = int(restart_marker_rows)
    if restart_marker_blocks:
        kw["restart_marker_blocks"] = int(restart_marker_blocks)
    im.save(buf, format="JPEG", **kw)
    return buf.getvalue()


def make_jpeg(seed: int, w: int, h: int, quality: int = 90, subsampling: str = "4:2:0",
              gray: bool = False, restart_marker_rows: int = 0) -> bytes:
    rng = np.random.default_rng(seed)
    return encode_jpeg(synth_pixels(rng, w, h, gray), quality, subsampling, restart_marker_rows)


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
    seed, (w, h, q, ss, gray), rst = args
    return make_jpeg(seed, w, h, q, ss, gray, rst)


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
                 workers: int = 1, restart_marker_rows: int = 0, lo: int = 0, hi: int | None = None) -> List[bytes]:
    """Images [lo, hi) of the logical n-image stream for `seed` (a rank's
    slice of a sharded corpus is generated without building the rest)."""
    spec = mixed_spec(seed, n, short_min, short_max)
    hi = n if hi is None else hi
    jobs = [(seed * 1_000_003 + i, spec[i], restart_marker_rows) for i in range(lo, hi)]
    if workers > 1:
        return _pool_map(jobs, workers)
    return [_make_one(j) for j in jobs]


def uniform_corpus(seed: int, n: int, w: int = 640, h: int = 480, quality: int = 90,
                   subsampling: str = "4:2:0", workers: int = 1) -> List[bytes]:
    jobs = [(seed * 1_000_003 + i, (w, h, quality, subsampling, False), 0) for i in range(n)]
    if workers > 1:
        return _pool_map(jobs, workers)
    return [_make_one(j) for j in jobs]
