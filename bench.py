#!/usr/bin/env python3
"""bench.py — device-resident JPEG decode + aspect-ratio-bucket resize, Mpixel/s.

Workload (BASELINE.json configs[1]): file-source-style synthetic JPEGs, mixed
aspect ratios (log-uniform [0.4, 2.5]), short side U[256, 2048], q U{75..95},
80/10/10 % 4:2:0/4:2:2/4:4:4, 5 % grayscale; buckets 1024/32/0.5/2.0.  The
logical stream (100k samples in the reference config) is drawn cyclically
from a seeded pool of unique images held in HBM; one step = one batch through
the whole decode + bucket + crop/resize path.  Coded bytes are resident in HBM
before timing starts; header parsing and batch planning on the host are
inside the timed region.

The logical stream: `--samples` file-source samples (100k for configs[1],
1M for configs[3] = `--workload cfg4`), sample s showing pool image
s % `--pool` (4,096 unique images for configs[1], 16,384 for configs[3]; the
pool's coded bytes, ~2.9 GB for 4,096, exceed the 256 MB Infinity Cache).

Multi-GPU: one process per GPU.  Under torchrun (the driver's N>1 launch)
RANK/WORLD_SIZE/LOCAL_RANK come from the environment; `python bench.py
--gpus N` without torchrun starts the N rank processes itself (this parent
never touches the GPU) with the same variables set.  Each rank decodes its
own contiguous slice of the logical stream (get_data_slice_multirank,
generator_files.rs:24-42) on device LOCAL_RANK (mod the device count: on a
1-GPU box the ranks share the card) with no data-path collective
("scaling": "weak"); only the barriers and the max-time reduction go over
torch.distributed (gloo).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--pool P] [--workload jpeg|cfg4|wds|png]
"""
from __future__ import annotations

import argparse
import json
import math
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
VALU_PEAK_T = 256 * 4 * 2.4e9 / 2 / 1e12  # VALU wave-instructions/s: 256 CUs x 4 SIMDs, one per 2 cycles, 2.4 GHz


# dg_submit* host phases (stats "host_us_<phase>"; the last is the wait for a free slot)
HOST_PHASES = ("plan", "pools", "layout", "lists", "upload", "h2d", "launch", "slotwait")


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--hw-queues", type=int, default=0,
                    help="GPU_MAX_HW_QUEUES for this process and its ranks (0: leave the runtime's default; <= 32)")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--windows", type=int, default=5,
                    help="timed windows of --steps steps each (SURVEY §8(d): the line reports the median window, "
                         "the others beside it as the spread)")
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=0, help="images per step (0: 256, or 1024 for wds's ImageNet-size JPEGs)")
    ap.add_argument("--pool", type=int, default=0,
                    help="unique images in the logical pool (0: 4096 for jpeg, 16384 for cfg4, 256 per rank for png)")
    ap.add_argument("--samples", type=int, default=0,
                    help="logical stream length sharded over ranks (0: 100000 for jpeg, 1000000 for cfg4)")
    ap.add_argument("--short-min", type=int, default=256)
    ap.add_argument("--short-max", type=int, default=2048)
    ap.add_argument("--size", type=int, default=0, help="bucket default_image_size (0: 1024, or 512 for wds)")
    ap.add_argument("--ratio", type=int, default=0, help="bucket downsampling_ratio (0: 32, or 16 for wds)")
    ap.add_argument("--sub-bits", type=int, default=0)
    ap.add_argument("--workers", type=int, default=0, help="corpus generation processes")
    ap.add_argument("--lead-bits", type=int, default=-1, help="entropy lead-in bits (-1 = library default)")
    ap.add_argument("--serial-steps", type=int, default=5,
                    help="untimed batches run one at a time after the timed region: per-kernel times without "
                         "the overlap of consecutive batches (roofline_isolated); 5, the batches the "
                         "isolated-pass kernel trace (tools/gpu_calib.sh ISO, SERIAL=5) measures: the entropy "
                         "stages differ by up to 30% between batches of different images")
    ap.add_argument("--pmc-json", default=os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "r06",
                                                       "pmc", "pmc_traffic.json"),
                    help="per-stage HBM bytes from a PMC run of this configuration (tools/pmc_traffic.py)")
    ap.add_argument("--wg-timing", action="store_true", help="debug: per-workgroup timing of the entropy kernels")
    ap.add_argument("--inflight", type=int, default=0,
                    help="batches in flight (context slots / output arenas); 0 = 4 for jpeg (3 vs 4: 94.6 vs 96.8 "
                         "Gpx/s mean of 3 alternating runs, profiles/r03/slots), 2 for wds, 4 for png (its inflate "
                         "chains leave most of the GPU idle: 2347 -> 2958 Mpx/s measured)")
    ap.add_argument("--entropy-once", type=int, default=-1, help="decode-once entropy staging (-1 = library default)")
    ap.add_argument("--entropy-lpt", type=int, default=-1, help="slow entropy workgroups first (-1 = library default)")
    ap.add_argument("--hb-bands", type=int, default=0, help="band H kernel: 8-row bands per workgroup (0 = default)")
    ap.add_argument("--ckpt", type=int, default=-1, help="entropy checkpoints (-1 = library default)")
    ap.add_argument("--idct-fused", type=int, default=-1, help="IDCT inside the entropy write kernel (-1 = default)")
    ap.add_argument("--decode-semantics", type=int, default=1, choices=(0, 1),
                    help="JPEG pixel semantics: 1 zune-jpeg 0.5.12 restated (default: the reference's decoder, the "
                         "mode INTEGRATION.md sets for the drop-in), 0 libjpeg-turbo (pinned to PIL)")
    ap.add_argument("--cpu-seconds", type=float, default=8.0, help="wall seconds of the CPU-baseline sample (x cores of CPU work)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--e2e-steps", type=int, default=3, help="host-memory (PCIe-inclusive) steps")
    ap.add_argument("--one-threads", type=int, default=32,
                    help="integration path: host threads calling dg_decode_one (coalesced into GPU batches); 0 = off")
    ap.add_argument("--one-images", type=int, default=0, help="images through dg_decode_one (0: 8 batches)")
    ap.add_argument("--ctx-opt", action="append", default=[],
                    help="extra context option key=value (experiments; repeatable)")
    ap.add_argument("--prog-lanes", type=int, default=-1,
                    help="context option prog_lanes: progressive batches in flight beside the baseline ones "
                         "(dg_decode_one coalescing; -1 = library default)")
    ap.add_argument("--shards", type=int, default=8, help="wds workload: shards of 1000 samples")
    ap.add_argument("--workload", choices=("jpeg", "cfg4", "png", "wds"), default="jpeg",
                    help="jpeg: configs[1] (the headline); cfg4: configs[3] (1M samples over a 16,384-image pool, "
                         "seed 4, sharded over the ranks); png: configs[4]-style RGB PNG + aligned L8 mask pairs "
                         "(decode + bucket-resize; the mask is forced to the image's bucket, worker_http.rs:186-214)")
    ap.add_argument("--encode", action="store_true",
                    help="pre_encode_images with encode_format jpeg, quality 92 (configs[4]: every payload "
                         "re-encoded on the GPU, WebDataset semantics worker_wds.rs:47-52)")
    ap.add_argument("--hv-fused", type=int, default=-1, help="fused first H + V pass (-1 = library default)")
    ap.add_argument("--rst-rows", type=int, default=0,
                    help="jpeg workload: the twin pool with a restart marker every N MCU rows (SURVEY §8(d); "
                         "not the headline config)")
    ap.add_argument("--progressive-frac", type=float, default=0.0,
                    help="jpeg workload: share of the pool written as progressive JPEGs (not the headline config)")
    ap.add_argument("--no-prog-split", action="store_true",
                    help="progressive-frac runs: dg_wait every batch whole (no dg_wait_ready / deferred completion)")
    ap.add_argument("--prog-ring", type=int, default=8192,
                    help="progressive-frac runs: output slots for progressive members awaiting completion")
    ap.add_argument("--max-device-mb", type=int, default=0,
                    help="context option max_device_mb: device memory budget per rank (0: none; batches that do "
                         "not fit are split)")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    if a.pool <= 0:
        a.pool = {"jpeg": 4096, "cfg4": 16384, "png": 256, "wds": 0}[a.workload]
    if a.samples <= 0:
        a.samples = 1_000_000 if a.workload == "cfg4" else 100_000
    if a.inflight <= 0:
        a.inflight = 4 if a.workload in ("png", "jpeg", "cfg4") else 2
    if a.batch <= 0:
        a.batch = 1024 if a.workload == "wds" else 256
    if a.size <= 0:  # BASELINE.json configs[2]: "decode + resize to 512"
        a.size = 512 if a.workload == "wds" else 1024
    if a.ratio <= 0:
        a.ratio = 16 if a.workload == "wds" else 32
    return a


def host_cores() -> tuple[int, str]:
    """The worker count the reference's runtime would pick: num_cpus::get()
    (worker_files.rs:86,151), i.e. the CPUs this process may run on, capped by
    a cgroup CPU quota -- and by the box's CPU share where the harness states
    one (OMP_NUM_THREADS: 16 per GPU on the MI355X boxes), so the pool never
    oversubscribes the cores it was given."""
    try:
        aff = len(os.sched_getaffinity(0))
    except Exception:
        aff = os.cpu_count() or 1
    n, basis = aff, [f"affinity {aff}"]
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            n = min(n, max(1, int(q) // int(per)))
            basis.append(f"cgroup quota {int(q) / int(per):g}")
    except (OSError, ValueError):
        pass
    share = os.environ.get("OMP_NUM_THREADS", "")
    if share.isdigit() and int(share) > 0:
        n = min(n, int(share))
        basis.append(f"CPU share (OMP_NUM_THREADS) {share}")
    return max(1, n), ", ".join(basis)


def cpu_share() -> int:
    return host_cores()[0]


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def reference_toolchain() -> str:
    """Probe for the reference's own toolchain: with cargo and
    the crates present, the Rust path itself would be the CPU baseline."""
    try:
        r = subprocess.run(["cargo", "--version"], capture_output=True, text=True, timeout=20)
        return (r.stdout or r.stderr).strip() or f"cargo exit {r.returncode}"
    except FileNotFoundError:
        return "cargo: not found (no Rust toolchain; the reference's crates are not vendored either)"
    except (OSError, subprocess.SubprocessError) as e:
        return f"cargo probe failed: {e}"


# --------------------------------------------------------------- CPU baseline

def _cpu_work(args):
    from oracle import oracle as O
    data, tw, th, enc, sem = args
    t = time.perf_counter()
    with O.semantics(sem):
        st, dec = O.decode_any(data)
    out = O.crop_and_resize(dec, tw, th, O.MODE_FIR) if (dec.shape[1], dec.shape[0]) != (tw, th) else dec
    if enc:
        O.jpeg_encode(out, 92)
    return dec.shape[0] * dec.shape[1], time.perf_counter() - t


def _pil_work(args):
    """Pillow proxy of the reference's per-sample work: decode, then the two
    Lanczos calls of crop_and_resize (image_processing.rs:288-323): the
    full-image resize to the scaled size and the crop box as a second resize."""
    import io as _io

    from PIL import Image

    from oracle import buckets as B
    data, tw, th, enc = args
    im = Image.open(_io.BytesIO(data))
    im.load()
    w, h = im.size
    if (w, h) != (tw, th):
        nw, nh = B.scaled_size(w, h, tw, th)
        l, t, bw, bh = B.fit_crop_box(nw, nh, tw, th)
        im = im.resize((nw, nh), Image.LANCZOS).resize((tw, th), Image.LANCZOS, box=(l, t, l + bw, t + bh))
    if enc:
        im.save(_io.BytesIO(), format="JPEG", quality=92)
    return w * h


def pillow_baseline(pool, targets, seconds: float, encode: bool = False):
    """The same bounded sample through Pillow 12 (libjpeg-turbo decode +
    Pillow's Lanczos convolution), one image per task on every host core."""
    import multiprocessing as mp
    cores, basis = host_cores()
    t = time.perf_counter()
    px = _pil_work((pool[0], *targets[0], encode))
    per_px = (time.perf_counter() - t) / max(px, 1)
    mean_px = np.mean([w * h for (w, h) in [image_dims(d)[:2] for d in pool[:32]]])
    n = int(max(cores, min(64 * len(pool), seconds * cores / max(per_px * mean_px, 1e-9))))
    jobs = [(pool[i % len(pool)], *targets[i % len(pool)], encode) for i in range(n)]
    p = mp.get_context("fork").Pool(cores)
    try:
        p.map(_pil_work, jobs[:cores], chunksize=1)
        t0 = time.perf_counter()
        res = p.map(_pil_work, jobs, chunksize=1)
        wall = time.perf_counter() - t0
    finally:
        p.close()
        p.join()
    tot = sum(res)
    return {"value": round(tot / wall / 1e6, 2), "unit": "Mpixel/s", "cores": cores, "kind": "pillow-proxy",
            "sample": f"{n} images of the same pool ({tot / 1e6:.1f} Mpx): PIL decode + resize(LANCZOS) to the "
                      f"scaled size + crop box resize(LANCZOS, box=){' + JPEG q92 save' if encode else ''}, "
                      f"{cores} processes ({basis}), {wall:.1f} s"}


def cpu_baseline(pool, targets, seconds: float, encode: bool = False, sem: int = 1):
    """Oracle (scalar C restatement of the reference path: decode +
    crop_and_resize, in the GPU run's decode semantics) on the host cores, one
    image per task like the reference's tokio worker (worker_files.rs:74-141)."""
    import multiprocessing as mp
    from oracle import oracle as O
    O.lib()
    cores, basis = host_cores()
    # size the sample from a one-image probe so the run takes ~`seconds`
    px, dt = _cpu_work((pool[0], *targets[0], encode, sem))
    per_px = dt / max(px, 1)
    mean_px = np.mean([w * h for (w, h) in [image_dims(d)[:2] for d in pool[:32]]])
    n = int(max(cores, min(64 * len(pool), seconds * cores / max(per_px * mean_px, 1e-9))))
    jobs = [(pool[i % len(pool)], *targets[i % len(pool)], encode, sem) for i in range(n)]
    p = mp.get_context("fork").Pool(cores)
    try:
        p.map(_cpu_work, jobs[:cores], chunksize=1)  # workers up and the oracle loaded
        t0 = time.perf_counter()
        res = p.map(_cpu_work, jobs, chunksize=1)
        wall = time.perf_counter() - t0
    finally:
        p.close()
        p.join()
    tot_px = sum(r[0] for r in res)
    return {"value": round(tot_px / wall / 1e6, 2), "unit": "Mpixel/s", "cores": cores, "kind": "port",
            "sample": f"{n} images of the same pool ({tot_px / 1e6:.1f} Mpx) through oracle/ (scalar C "
                      f"decode in {'zune-jpeg' if sem else 'libjpeg-turbo'} semantics + FIR-mode Lanczos3 "
                      f"crop_and_resize{' + JPEG q92 encode' if encode else ''}), "
                      f"{cores} processes ({basis}), {wall:.1f} s",
            "cpu_model": cpu_model(), "reference_toolchain": reference_toolchain()}


def image_dims(data: bytes):
    """(w, h, decoded channels) from the header (oracle helpers: bench plumbing)."""
    from oracle import oracle as O
    if data[:8] == b"\x89PNG\r\n\x1a\n":
        st, w, h, c = O.png_info(data)[:4]
        return w, h, c
    return tuple(O.jpeg_info(data)[1:4])


def png_stage_bytes(data: bytes, dim, target) -> dict:
    """Algorithmic bytes per stage for one PNG: inflate reads the zlib stream
    and writes the filtered scanlines; unfilter reads and writes them once;
    the resize passes as for a non-fused source of C channels."""
    from oracle import buckets as B
    from oracle import oracle as O
    w, h, c = dim
    tw, th = target
    info = O.png_info(data)
    depth, ctype = info[4], info[5]
    spp = {0: 1, 2: 3, 3: 1, 4: 2, 6: 4}[ctype]
    rb = (spp * depth * w + 7) // 8
    b = {"png_inflate": len(data) + h * (rb + 1), "png_unfilter": h * (rb + 1) + h * rb,
         "resize_h1": 0.0, "resize_v1": 0.0, "resize_h2": 0.0, "resize_v2": 0.0, "copy": 0.0}
    if (w, h) != (tw, th):
        nw, nh = B.scaled_size(w, h, tw, th)
        l, t, bw, bh = B.fit_crop_box(nw, nh, tw, th)
        fold_x = abs(l - round(l)) <= 1e-6 and abs(bw - tw) <= 1e-6
        fold_y = abs(t - round(t)) <= 1e-6 and abs(bh - th) <= 1e-6
        cw, ch = w, h
        if nw != w:
            wx = tw if fold_x else nw
            b["resize_h1"] = c * (w * h + wx * h)
            cw = wx
        elif fold_x:
            cw = tw
        if nh != h:
            hy = th if fold_y else nh
            b["resize_v1"] = c * (cw * h + cw * hy)
            ch = hy
        elif fold_y:
            ch = th
        if not fold_x:
            b["resize_h2"] = c * (cw * ch + tw * ch)
            cw = tw
        if not fold_y:
            b["resize_v2"] = c * (cw * ch + cw * th)
    else:
        b["copy"] = 2 * c * w * h
    return b


def png_pair(args):
    """One configs[4] sample: an RGB PNG (PIL encoder: adaptive filters, zlib
    level 6) and an L8 mask PNG of the same size (seed 5 stream)."""
    from datago_amd import synth
    seed, (w, h, _, _, _) = args
    rng = np.random.default_rng(seed)
    img = synth.pil_png(synth.synth_pixels(rng, w, h))
    yy, xx = np.mgrid[0:h, 0:w]
    cx, cy, r = rng.uniform(0.3, 0.7) * w, rng.uniform(0.3, 0.7) * h, rng.uniform(0.2, 0.45) * min(w, h)
    mask = (((xx - cx) ** 2 + (yy - cy) ** 2) < r * r).astype(np.uint8) * 255
    return img, synth.pil_png(mask)


def png_corpus(seed: int, n: int, short_min: int, short_max: int, workers: int, lo: int, hi: int):
    from datago_amd import synth
    spec = synth.mixed_spec(seed, n, short_min, short_max)
    jobs = [(seed * 1_000_003 + i, spec[i]) for i in range(lo, hi)]
    if workers > 1:
        import multiprocessing as mp
        p = mp.get_context("fork").Pool(workers)
        try:
            pairs = p.map(png_pair, jobs, chunksize=1)
        finally:
            p.close()
            p.join()
    else:
        pairs = [png_pair(j) for j in jobs]
    out = []
    for img, mask in pairs:
        out += [img, mask]
    return out


# ------------------------------------------------------------- roofline

def pmc_config_key(a) -> str:
    """Identifies the workload a PMC traffic file was measured on."""
    return f"batch={a.batch} pool={a.pool} size={a.size}/{a.ratio} short={a.short_min}-{a.short_max}"


def band_dec_takes(w: int, nw: int) -> bool:
    """Mirrors band_dec_mode (pipeline.cpp): k_band_dec runs the first H pass
    W -> nw when the 128-column tile's segment fits 640 pixels and every
    16-column subtile's window two 64-wide K steps."""
    scale = w / nw
    fs = max(scale, 1.0)
    ksize = math.ceil(3.0 * fs) * 2 + 1
    span = math.ceil(127 * scale + 6.0 * fs) + 2 + 8 + ksize + 8 + 16
    window = 15 + math.ceil(15 * scale) + ksize + 2
    return (span <= 320 and window <= 64) or (span <= 640 and window <= 128)


def stage_bytes(L, data: bytes, dim, target, band_dec: bool = True) -> dict:
    """Algorithmic bytes each kernel stage must move for one image (DESIGN.md
    §Roofline): its minimal input + output, intermediates counted once.  With
    k_band_dec the first H pass reads the coefficients (128 B per block) and
    writes the H intermediate: no planes in between."""
    from oracle import buckets as B
    w, h, nc = dim
    tw, th = target
    st, info = L.probe(data)
    S = len(data)
    if nc == 1:
        nblk = ((w + 7) // 8) * ((h + 7) // 8)
    else:
        hm = max(info.h_samp[:3]); vm = max(info.v_samp[:3])
        mcus = -(-w // (8 * hm)) * -(-h // (8 * vm))
        nblk = mcus * sum(info.h_samp[c] * info.v_samp[c] for c in range(3))
    b = {"destuff": 2 * S, "huff_sync": S, "huff_fix": 0.0, "huff_scan": 0.0,
         "huff_write": S + 128 * nblk, "idct": 128 * nblk + 64 * nblk,
         "color": (64 * nblk + 3 * w * h) if nc == 3 else 0.0, "coeffs": 0.0,
         "resize_h1": 0.0, "resize_v1": 0.0, "resize_h2": 0.0, "resize_v2": 0.0, "copy": 0.0}
    if (w, h) != (tw, th):
        # mirrors the pass plan in pipeline.cpp: integral crop offsets fold into call 1
        nw, nh = B.scaled_size(w, h, tw, th)
        l, t, bw, bh = B.fit_crop_box(nw, nh, tw, th)
        fold_x = abs(l - round(l)) <= 1e-6 and abs(bw - tw) <= 1e-6
        fold_y = abs(t - round(t)) <= 1e-6 and abs(bh - th) <= 1e-6
        cw, ch = w, h
        if nw != w:
            wx = tw if fold_x else nw
            if band_dec and band_dec_takes(w, nw):  # k_band_dec: coefficients in, H intermediate out
                b["resize_h1"] = 128 * nblk + nc * wx * h
                b["idct"] = 0.0
                b["color"] = 0.0
            elif nc == 3:  # fused: upsample + colour from the planes inside the first H pass
                b["resize_h1"] = b["color"] - 3 * w * h + nc * wx * h
                b["color"] = 0.0
            else:
                b["resize_h1"] = nc * (w * h + wx * h)
            cw = wx
        elif fold_x:
            cw = tw
        if nh != h:
            hy = th if fold_y else nh
            b["resize_v1"] = nc * (cw * h + cw * hy)
            ch = hy
        elif fold_y:
            ch = th
        if not fold_x:
            b["resize_h2"] = nc * (cw * ch + tw * ch)
            cw = tw
        if not fold_y:
            b["resize_v2"] = nc * (cw * ch + cw * th)
    else:
        b["copy"] = 2 * nc * w * h
    return b


# ------------------------------------------------------------------- ranks

def _free_port() -> int:
    with socket.socket() as s_:
        s_.bind(("127.0.0.1", 0))
        return s_.getsockname()[1]


def launch_ranks(n: int) -> int:
    """`--gpus N` without torchrun: start N rank processes of this script
    (RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* set before they start; this parent
    imports no GPU runtime), stream their output, and return the worst exit
    code.  If a rank fails, the others are stopped (they would wait forever
    at the next barrier)."""
    env = dict(os.environ, WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(_free_port()))
    procs = [subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:],
                              env=dict(env, RANK=str(r), LOCAL_RANK=str(r))) for r in range(n)]
    rc = 0
    try:
        while procs:
            for p_ in list(procs):
                code = p_.poll()
                if code is None:
                    continue
                procs.remove(p_)
                if code != 0:
                    rc = rc or code
                    for q in procs:
                        q.terminate()
            time.sleep(0.2)
    finally:
        for q in procs:
            q.kill()
    return rc


def jpeg_pool(a, rank: int, world: int, workers: int, dist):
    """The rank's slice of the logical stream and the pool images it shows.

    Sample s of the `a.samples`-long stream shows pool image s % a.pool (the
    stream cycles over the pool); rank r owns the contiguous
    slice get_data_slice_multirank(a.samples, r, world) and step k of the
    run decodes its samples lo + (k*B + j) mod (hi - lo).  Pool images are
    generated once per machine into a cache shared by the ranks (each rank
    makes a 1/world share of what any rank needs, then all load theirs)."""
    from datago_amd import synth
    from datago_amd.sharding import get_data_slice_multirank
    seed = 4 if a.workload == "cfg4" else 2  # configs[1] seed 2, configs[3] seed 4
    nb = max(1, a.warmup) + a.steps

    def images_of(r):
        lo, hi = get_data_slice_multirank(a.samples, r, world)
        span = max(1, hi - lo)
        return [(lo + (k * a.batch + j) % span) % a.pool for k in range(nb) for j in range(a.batch)]

    union = sorted({i for r in range(world) for i in images_of(r)})
    t0 = time.perf_counter()
    made = synth.generate_pool_images(seed, a.pool, union[rank::world], workers, a.short_min, a.short_max,
                                      a.progressive_frac,
                                      progress=lambda m: print(f"[rank {rank}] {m}", file=sys.stderr, flush=True),
                                      restart_marker_rows=a.rst_rows)
    if world > 1:
        dist.barrier()
    mine = images_of(rank)
    uniq = sorted(set(mine))
    pos = {img: k for k, img in enumerate(uniq)}
    pool = synth.load_pool_images(seed, a.pool, uniq, a.short_min, a.short_max, a.progressive_frac,
                                  restart_marker_rows=a.rst_rows)
    seq = [pos[i] for i in mine]  # batch k = seq[k*B:(k+1)*B]
    lo, hi = get_data_slice_multirank(a.samples, rank, world)
    return pool, seq, (lo, hi), made, time.perf_counter() - t0


# ------------------------------------------------------------------- main

def pin_rank_cores(local: int, local_world: int):
    """Give each rank of this node a disjoint, contiguous share of the CPUs
    the job may use (before anything touches the GPU or starts threads): the
    ranks' host planning, Python loop and pool workers then never compete for
    a core, and contiguous ids keep a rank on one socket on the usual
    GPU-per-socket layouts.  DG_NO_PIN=1 disables it.  Returns the CPU list."""
    if local_world <= 1 or os.environ.get("DG_NO_PIN"):
        return None
    try:
        cpus = sorted(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        return None
    per = len(cpus) // local_world
    if per < 1:
        return None
    mine = cpus[local * per:(local + 1) * per]
    try:
        os.sched_setaffinity(0, mine)
    except OSError:
        return None
    return mine


def main() -> int:
    a = parse()
    if a.hw_queues > 0:  # before anything initialises HIP (ranks inherit it)
        os.environ["GPU_MAX_HW_QUEUES"] = str(min(a.hw_queues, 32))
    if "WORLD_SIZE" not in os.environ and a.gpus > 1:
        return launch_ranks(a.gpus)
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    pinned = pin_rank_cores(local, int(os.environ.get("LOCAL_WORLD_SIZE", str(world))))
    if world != a.gpus and rank == 0:
        print(f"bench.py: --gpus {a.gpus} but WORLD_SIZE={world}; measuring {world} ranks", file=sys.stderr)
    import torch
    import torch.distributed as dist
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    from datago_amd import _lib as L
    from datago_amd import synth
    from oracle import buckets as B

    from datago_amd.sharding import get_data_slice_multirank, max_over_ranks, sum_over_ranks
    workers = a.workers or cpu_share()
    t_gen = time.perf_counter()
    n_made = 0
    lo, hi = 0, 0
    png = a.workload == "png"
    wds = a.workload == "wds"
    tar_arena = None
    seq = None  # jpeg/cfg4: pool positions of the rank's stream, batch after batch
    if a.workload in ("jpeg", "cfg4"):
        pool, seq, (lo, hi), n_made, _ = jpeg_pool(a, rank, world, workers, dist)
    elif wds:  # configs[2]: WebDataset shards held in memory, indexed by dg_wds_index (zero-copy members)
        tars = [synth.make_wds_shard(3 * 1000 + k, 1000, first_key=1000 * k, workers=workers)
                for k in range(a.shards)]
        t_idx = time.perf_counter()
        tar_arena = np.frombuffer(b"".join(tars), np.uint8)
        members, base = [], 0
        for t_ in tars:  # this rank's samples (SipHash-1-3 of the key % world, generator_wds.rs:133-148)
            for smp in L.wds_index(t_, rank, world, "jpg"):
                members += [(base + off, n) for (name, off, n) in smp if name.endswith(".jpg")]
            base += len(t_)
        wds_index_s = time.perf_counter() - t_idx
        pool = [tar_arena[off:off + n].tobytes() for off, n in members]
    elif png:  # configs[4]: pairs (image, mask), seed 5; a.pool counts images (2 per pair)
        npair = max(1, a.pool // 2)
        plo, phi = get_data_slice_multirank(npair * world, rank, world)
        pool = png_corpus(5, npair * world, a.short_min, a.short_max, workers, plo, phi)
    t_gen = time.perf_counter() - t_gen
    ndev = torch.cuda.device_count()
    if ndev < 1:
        raise RuntimeError("bench.py needs a GPU (HIP device)")
    local = local % ndev  # more ranks than devices (a 1-GPU rehearsal of --gpus N): ranks share the card
    torch.cuda.set_device(local)
    tr = B.ARAwareTransform(a.size, a.ratio, 0.5, 2.0)
    dims = [image_dims(d) for d in pool]
    ctx = L.Context(local, crop_and_resize=True, default_image_size=a.size, downsampling_ratio=a.ratio,
                    min_aspect_ratio=0.5, max_aspect_ratio=2.0, pre_encode_images=a.encode, encode_format=1,
                    jpeg_quality=92)
    # multi-payload alignment (worker_wds.rs:68-76, worker_http.rs:186-214): every
    # payload after the first of a sample takes the first one's bucket
    forced_pool = [-1] * len(pool)
    if png:
        for i in range(1, len(pool), 2):
            forced_pool[i] = ctx.buckets.closest(dims[i - 1][0], dims[i - 1][1])
    targets = [tr.target_size(w, h) if f < 0 else ctx.buckets.get(f)[:2] for (w, h, _), f in zip(dims, forced_pool)]
    if a.sub_bits:
        ctx.set_option("sub_bits", a.sub_bits)
    if a.lead_bits >= 0:
        ctx.set_option("lead_bits", a.lead_bits)
    if a.wg_timing:
        ctx.set_option("wg_timing", 1)
    if a.hb_bands:
        ctx.set_option("hb_bands", a.hb_bands)
    ctx.set_option("decode_semantics", a.decode_semantics)
    if a.ckpt >= 0:
        ctx.set_option("ckpt", a.ckpt)
    if a.hv_fused >= 0:
        ctx.set_option("hv_fused", a.hv_fused)
    if a.idct_fused >= 0:
        ctx.set_option("idct_fused", a.idct_fused)
    if a.progressive_frac > 0:
        ctx.set_option("progressive", 1)
    if a.prog_lanes >= 0:
        ctx.set_option("prog_lanes", a.prog_lanes)
    for kv in a.ctx_opt:
        k_, v_ = kv.split("=", 1)
        ctx.set_option(k_, int(v_))
    if a.entropy_lpt >= 0:
        ctx.set_option("entropy_lpt", a.entropy_lpt)
    if a.entropy_once >= 0:
        ctx.set_option("entropy_once", a.entropy_once)
    ctx.set_option("slots", a.inflight)
    if a.max_device_mb > 0:
        ctx.set_option("max_device_mb", a.max_device_mb)
    # ---- pool -> HBM (one arena, 16-byte aligned entries; wds: the shards themselves)
    if wds:
        host_arena = np.concatenate([tar_arena, np.zeros(64, np.uint8)])
        offs = [off for off, _ in members]
        o = host_arena.nbytes
    else:
        offs, o = [], 0
        for d in pool:
            offs.append(o)
            o += (len(d) + 16 + 15) // 16 * 16
        host_arena = np.zeros(o, np.uint8)
        for d, of in zip(pool, offs):
            host_arena[of:of + len(d)] = np.frombuffer(d, np.uint8)
    d_arena = ctx.alloc(o)
    ctx.h2d(d_arena, host_arena)
    h_base = host_arena.ctypes.data
    if a.encode:  # caller buffers sized by the encoder bound (datago_hip.h dg_output_size)
        out_bytes = [ctx.output_size(d, f)[1] for d, f in zip(pool, forced_pool)]
    else:
        out_bytes = [tw * th * nc for (tw, th), (_, _, nc) in zip(targets, dims)]
    band_dec = "band_dec=1" in a.ctx_opt  # k_band_dec is off by default (library option band_dec)
    img_stage_bytes = [png_stage_bytes(d, dim, tgt) if png else stage_bytes(L, d, dim, tgt, band_dec)
                       for d, dim, tgt in zip(pool, dims, targets)]
    B_ = min(a.batch, 1 << 16)
    # output arena for one step (reused), sized for the largest B_ outputs
    # one arena per batch in flight: the B_ largest outputs (images repeat when
    # the batch is larger than the pool), each padded to 16 bytes
    reps = -(-B_ // len(pool))
    out_cap = sum(sorted(out_bytes * reps)[-B_:]) + 16 * B_
    d_out = [ctx.alloc(out_cap) for _ in range(a.inflight)]

    # per-image arrays: the loop below is harness bookkeeping around the library
    # calls, vectorised so that the caller's Python stays off the critical path
    n_pool = len(pool)
    offs_np = np.asarray(offs, np.uint64)
    lens_np = np.asarray([len(d) for d in pool], np.uint64)
    out_np = np.asarray(out_bytes, np.uint64)
    out_al_np = (out_np + 15) // 16 * 16
    forced_np = np.asarray(forced_pool, np.int32)

    def batch_idx(k: int):
        if seq is not None:
            k %= len(seq) // B_  # serial / e2e passes reuse the stream's batches
            return np.asarray(seq[k * B_:(k + 1) * B_], np.int64)
        return (k * B_ + np.arange(B_, dtype=np.int64)) % n_pool

    # Progressive members of a submission run in the library's progressive
    # aggregate (datago_hip.h dg_wait_ready): the loop waits for the other
    # members only (dg_wait_ready) and completes a batch's progressive members
    # later (dg_wait), so their outputs live in a ring of their own, reused
    # once the batch that held a slot is complete.  Everything is complete
    # before the timed region ends.
    split = a.progressive_frac > 0 and not a.no_prog_split
    prog_of = [synth.is_progressive_jpeg(d) for d in pool] if split else [False] * len(pool)
    prog_np = np.asarray(prog_of, bool)
    ring = {"next": 0, "owner": [], "done": set(), "deferred": []}
    if split:
        ring_sz = max([(out_bytes[i] + 15) // 16 * 16 for i in range(len(pool)) if prog_of[i]] or [16])
        ring["n"] = a.prog_ring
        ring["size"] = ring_sz
        ring["base"] = ctx.alloc(a.prog_ring * ring_sz)
        ring["owner"] = [-1] * a.prog_ring

    def submit(k: int):
        idx = batch_idx(k)
        slot = k % a.inflight  # one output arena per batch in flight
        if not prog_np[idx].any():
            al = out_al_np[idx]
            outs = np.uint64(d_out[slot]) + (np.cumsum(al) - al)
        else:
            outs, oo = [], 0
            for i in idx:
                if prog_of[i]:
                    r = ring["next"] % ring["n"]
                    ring["next"] += 1
                    while ring["owner"][r] >= 0 and ring["owner"][r] not in ring["done"]:
                        finish_deferred(ring["deferred"].pop(0))  # oldest first
                    ring["owner"][r] = k
                    outs.append(ring["base"] + r * ring["size"])
                else:
                    outs.append(d_out[slot] + oo)
                    oo += int(out_al_np[i])
            outs = np.asarray(outs, np.uint64)
        ticket, metas = ctx.submit_device(np.uint64(h_base) + offs_np[idx], np.uint64(d_arena) + offs_np[idx],
                                          lens_np[idx], outs, out_np[idx], forced_np[idx])
        return ticket, metas, idx, k

    def check(metas, idx, which=None):
        st = L.meta_status(metas)[:len(idx)]
        bad = np.nonzero((st != 0) if which is None else ((st != 0) & which[idx]))[0]
        if bad.size:
            j = int(bad[0])
            raise RuntimeError(f"image {int(idx[j])} status {int(st[j])}: {L.last_error()}")

    def complete(pend):
        ticket, metas, idx, k = pend
        ctx.wait(ticket)
        check(metas, idx)
        ring["done"].add(k)
        return idx

    def finish_deferred(pend, on_done=None):
        ticket, metas, idx, k = pend
        ctx.wait(ticket)
        check(metas, idx, prog_np)
        ring["done"].add(k)
        if on_done or ring.get("on_done"):
            (on_done or ring["on_done"])(idx[prog_np[idx]])

    def ready(pend):  # split mode: the batch's other members; its progressive ones later
        ticket, metas, idx, k = pend
        ctx.wait_ready(ticket)
        check(metas, idx, ~prog_np)
        if prog_np[idx].any():
            ring["deferred"].append(pend)
        else:
            ring["done"].add(k)
        return idx[~prog_np[idx]]

    host_s = {"submit": 0.0}

    def run(k0: int, n: int, on_done=None):
        pend = []  # batch k + inflight - 1 is submitted before batch k is waited on
        done_fn = ready if split else complete
        ring["on_done"] = on_done
        for k in range(k0, k0 + n):
            ts = time.perf_counter()
            pend.append(submit(k))
            host_s["submit"] += time.perf_counter() - ts
            if len(pend) >= a.inflight:
                idx = done_fn(pend.pop(0))
                if on_done:
                    on_done(idx)
        while pend:
            idx = done_fn(pend.pop(0))
            if on_done:
                on_done(idx)
        while ring["deferred"]:
            finish_deferred(ring["deferred"].pop(0))

    run(0, max(1, a.warmup))
    host_s["submit"] = 0.0
    ctx.set_option("reset_host_us", 1)
    # ---- timed region
    ctx.set_option("timing", 1)
    stage_tot = {}
    stage_alg = {}
    acc = {"px": 0, "alg": 0.0, "coded": 0, "outpx": 0}

    stage_keys = sorted({kk for sb in img_stage_bytes for kk in sb})
    stage_mat = np.asarray([[sb.get(kk, 0.0) for kk in stage_keys] for sb in img_stage_bytes], np.float64)
    px_np = np.asarray([w * h for (w, h, _) in dims], np.int64)
    outpx_np = np.asarray([tw * th for (tw, th) in targets], np.int64)
    alg_np = np.asarray([len(d) + nc * w * h + nc * tw * th  # SURVEY §8(d) B_alg
                         for d, (w, h, nc), (tw, th) in zip(pool, dims, targets)], np.float64)

    def on_done(idx):
        idx = np.asarray(idx, np.int64)
        if idx.size:
            for kk, vv in zip(stage_keys, stage_mat[idx].sum(0)):
                stage_alg[kk] = stage_alg.get(kk, 0.0) + float(vv)
            acc["px"] += int(px_np[idx].sum())
            acc["coded"] += int(lens_np[idx].sum())
            acc["alg"] += float(alg_np[idx].sum())
            acc["outpx"] += int(outpx_np[idx].sum())
        for name, ms in ctx.timings().items():
            stage_tot[name] = stage_tot.get(name, 0.0) + ms

    # K timed steps per window, --windows windows back to back (each bracketed by a barrier and a device
    # sync on both sides); the line reports the median window over ranks' max times
    nwin = max(1, a.windows)
    win = []  # per window: (dt, px, alg, outpx) of this rank
    k_next = max(1, a.warmup)
    for w_ in range(nwin):
        acc0 = dict(acc)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        ctx.synchronize()
        t0 = time.perf_counter()
        run(k_next, a.steps, on_done)
        ctx.synchronize()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        dt_w = time.perf_counter() - t0
        k_next += a.steps
        win.append((dt_w, acc["px"] - acc0["px"], acc["alg"] - acc0["alg"], acc["outpx"] - acc0["outpx"]))
    steps_all = a.steps * nwin
    ctx.set_option("timing", 0)
    # host planning phases of the timed steps only (read before the untimed legs add to them)
    host_phases = {q: round(ctx.stat("host_us_" + q) / 1e3 / steps_all, 3)
                   for q in HOST_PHASES}
    host_phases_cpu = {q: round(ctx.stat("host_cpu_us_" + q) / 1e3 / steps_all, 3)
                       for q in HOST_PHASES[:-1]}
    ph_all = sum_over_ranks([host_phases[q] if r == rank else 0.0 for r in range(world)
                             for q in HOST_PHASES] +
                            [host_phases_cpu[q] if r == rank else 0.0 for r in range(world)
                             for q in HOST_PHASES[:-1]], world)
    # per window: max time over ranks, totals over ranks; the median window by rate
    win_dt = max_over_ranks([w_[0] for w_ in win], world)
    win_sum = sum_over_ranks([float(w_[j]) for w_ in win for j in (1, 2, 3)], world)
    win_rate = [win_sum[3 * j] / win_dt[j] / 1e6 for j in range(nwin)]
    med = sorted(range(nwin), key=lambda j: win_rate[j])[nwin // 2]
    dt, dt_max = win[med][0], win_dt[med]
    px_all, alg_all, outpx_all = win_sum[3 * med], win_sum[3 * med + 1], win_sum[3 * med + 2]
    alg_bytes = win[med][2]
    per_rank_s = sum_over_ranks([dt if r == rank else 0.0 for r in range(world)], world)
    # host CPU time each rank spent planning + submitting its batches (the 8-GPU host budget)
    per_rank_host = sum_over_ranks([host_s["submit"] / nwin if r == rank else 0.0 for r in range(world)], world)

    # ---- isolated per-kernel times: batches one at a time (untimed, reported only)
    ser_tot, ser_alg, ser_n = {}, {}, 0
    if a.serial_steps > 0:
        ctx.set_option("timing", 1)
        for k in range(a.serial_steps):
            idx = complete(submit(k))
            ser_n += 1
            for i in idx:
                for kk, vv in img_stage_bytes[i].items():
                    ser_alg[kk] = ser_alg.get(kk, 0.0) + vv
            for name, ms in ctx.timings().items():
                ser_tot[name] = ser_tot.get(name, 0.0) + ms
        ctx.set_option("timing", 0)

    # ---- end-to-end (host memory in and out: PCIe-inclusive), reported only
    e2e = e2e_dev = e2e_sync = d2h = None
    if a.e2e_steps > 0 and rank == 0:
        # pinned D2H bandwidth of this box (the host-out path's ceiling): best of 3 copies of 1 GiB
        try:
            xs_ = torch.empty(1 << 30, dtype=torch.uint8, device="cuda")
            hs_ = torch.empty(1 << 30, dtype=torch.uint8).pin_memory()
            best = None
            for _ in range(3):
                torch.cuda.synchronize()
                t_ = time.perf_counter()
                hs_.copy_(xs_, non_blocking=True)
                torch.cuda.synchronize()
                t_ = time.perf_counter() - t_
                best = t_ if best is None else min(best, t_)
            d2h = (1 << 30) / best / 1e9
            del xs_, hs_
        except RuntimeError:
            pass
        # synchronous host-in / host-out batches into fresh arrays (dg_submit + dg_wait per call)
        t1 = time.perf_counter()
        e2e_px = 0
        for k in range(a.e2e_steps):
            idx = batch_idx(k)
            res = ctx.decode_batch([pool[i] for i in idx], [forced_pool[i] for i in idx])
            e2e_px += sum(dims[i][0] * dims[i][1] for i, r in zip(idx, res) if r[0] == 0)
        e2e_sync = e2e_px / (time.perf_counter() - t1) / 1e6
        # the loader's steady state: a reused, page-locked output pool (dg_host_register), batches
        # pipelined (batch k + inflight - 1 submitted before batch k is waited on); outputs DMA'd from
        # HBM straight into the pool
        n_e2e = max(a.e2e_steps, 2 * a.inflight)
        arenas = []
        for _ in range(a.inflight):
            ar = np.zeros(out_cap, np.uint8)
            ctx.host_register(ar)
            arenas.append(ar)
        direct0 = ctx.stat("direct_d2h")

        def host_submit(k):
            idx = batch_idx(k)
            ar, oo, outs_ = arenas[k % a.inflight], 0, []
            for i in idx:
                outs_.append(ar[oo:oo + out_bytes[i]])
                oo += (out_bytes[i] + 15) // 16 * 16
            tk, ms_, keep = ctx.submit_host([pool[i] for i in idx], outs_, [forced_pool[i] for i in idx])
            return tk, ms_, keep, idx

        t1 = time.perf_counter()
        e2e_px, e2e_out, pend = 0, 0, []
        for k in range(n_e2e):
            pend.append(host_submit(k))
            if len(pend) >= a.inflight or k == n_e2e - 1:
                while pend and (len(pend) >= a.inflight or k == n_e2e - 1):
                    tk, ms_, keep, idx = pend.pop(0)
                    ctx.wait(tk)
                    for j, i in enumerate(idx):
                        if ms_[j].status == 0:
                            e2e_px += dims[i][0] * dims[i][1]
                            e2e_out += ms_[j].nbytes
        dt_e2e = time.perf_counter() - t1
        e2e = e2e_px / dt_e2e / 1e6
        e2e_direct = ctx.stat("direct_d2h") - direct0
        e2e_out_gbs = e2e_out / dt_e2e / 1e9
        for ar in arenas:
            ctx.host_unregister(ar)
        # host coded bytes in -> HBM tensors out (the training-loop hand-off: PCIe carries the
        # compressed stream only)
        t1 = time.perf_counter()
        e2e_px = 0
        for k in range(a.e2e_steps):
            idx = batch_idx(k)
            res = ctx.decode_batch_torch([pool[i] for i in idx], [forced_pool[i] for i in idx])
            e2e_px += sum(dims[i][0] * dims[i][1] for i, r in zip(idx, res) if r[0] == 0)
            del res
        e2e_dev = e2e_px / (time.perf_counter() - t1) / 1e6

    # ---- integration path (INTEGRATION.md GpuImageStage::payload): dg_decode_one from many host threads,
    # the library coalescing concurrent calls into GPU batches (coalesce_max 64, coalesce_us 500); host in ->
    # host out like e2e_host_mpix_s, reported only
    one = None
    if a.one_threads > 0 and rank == 0 and not a.encode:
        import itertools
        import threading
        n_one = a.one_images or 8 * B_  # ~0.3 s of calls: 512 measured only ~0.07 s and varied run to run
        order = [i for k in range(-(-n_one // B_)) for i in batch_idx(k)][:n_one]
        ctx.decode_one(pool[order[0]], forced_pool[order[0]])  # warm the single-image path
        b0, i0 = ctx.stat("coalesced_batches"), ctx.stat("coalesced_images")
        ctr = itertools.count()
        done_px = [0] * a.one_threads
        fails = [0] * a.one_threads

        # one reused, page-locked output buffer per calling thread (the glue's payload buffers)
        one_bufs = [np.zeros(max(out_bytes), np.uint8) for _ in range(a.one_threads)]
        for ob_ in one_bufs:
            ctx.host_register(ob_)

        def one_worker(t):
            while True:
                j = next(ctr)
                if j >= n_one:
                    return
                i = order[j]
                st_, _, _ = ctx.decode_one(pool[i], forced_pool[i], out=one_bufs[t])
                if st_ == 0:
                    done_px[t] += dims[i][0] * dims[i][1]
                else:
                    fails[t] += 1

        ths = [threading.Thread(target=one_worker, args=(t,)) for t in range(a.one_threads)]
        t1 = time.perf_counter()
        for th in ths:
            th.start()
        for th in ths:
            th.join()
        dt1 = time.perf_counter() - t1
        for ob_ in one_bufs:
            ctx.host_unregister(ob_)
        nb_ = ctx.stat("coalesced_batches") - b0
        one = {"threads": a.one_threads, "images": n_one, "failed": sum(fails),
               "mpix_s": round(sum(done_px) / dt1 / 1e6, 2), "images_per_s": round(n_one / dt1, 1),
               "gpu_batches": nb_, "mean_images_per_batch": round((ctx.stat("coalesced_images") - i0) / max(nb_, 1), 1),
               "coalesce_max": 64, "coalesce_us": 500, "coalesce_inflight": ctx.stat("coalesce_inflight"),
               "prog_lanes": a.prog_lanes,
               "note": "host JPEG bytes in -> host RGB out per call (PCIe both ways) into a reused page-locked "
                       "buffer per thread (dg_host_register), like e2e_host_mpix_s"}
        # the same calls from native threads (tools/one_bench, linked to the library): the Rust glue's
        # tokio workers are native; Python threads also contend for the interpreter lock between calls
        native = os.path.join(ROOT, "tools", "one_bench")
        if os.path.exists(native) and all(forced_pool[i] < 0 for i in order):
            import struct
            import subprocess
            import tempfile
            with tempfile.NamedTemporaryFile(prefix="one_pool_", suffix=".bin", delete=False) as tf:
                tf.write(struct.pack("<I", len(order)))
                for i in order:
                    tf.write(struct.pack("<Q", len(pool[i])))
                    tf.write(pool[i])
            try:
                r = subprocess.run([native, tf.name, str(a.one_threads), str(len(order)), str(a.size), str(a.ratio),
                                    str(a.decode_semantics)] + list(a.ctx_opt),
                                   capture_output=True, text=True, timeout=300)
                one["native_threads"] = (json.loads(r.stdout.strip().splitlines()[-1]) if r.returncode == 0 else
                                         {"error": r.returncode, "stderr": r.stderr[-300:]})
            except (subprocess.TimeoutExpired, ValueError, IndexError) as e:
                one["native_threads"] = {"error": str(e)[:200]}
            finally:
                os.unlink(tf.name)

    result = None
    if rank == 0:
        steps = steps_all  # stage spans are summed over every window
        # dominant kernel (by time) and its algorithmic bytes per launch
        kern = {k: v for k, v in stage_tot.items() if k not in ("upload", "download")}
        dom = max(kern, key=kern.get)
        dom_ms = kern[dom] / steps
        per_step_alg = alg_bytes / a.steps  # the median window's
        dom_alg = stage_alg[dom] / steps if dom in stage_alg else 0.0
        achieved = dom_alg / (dom_ms / 1e3) / 1e9 if dom_ms > 0 else 0.0
        gpu_ms = sum(kern.values()) / steps
        iso = None
        if ser_n:
            skern = {k: v / ser_n for k, v in ser_tot.items() if k not in ("upload", "download")}
            # the dominant kernel is the one with the largest share of the timed region's stage spans
            # (resize_h1: ~6 of 18 ms per step); its duration is the isolated pass's (the entropy sync
            # kernel's isolated time is as long, but it keeps its speed beside the other batches)
            sdom = dom if dom in skern else max(skern, key=skern.get)
            sach = (ser_alg.get(sdom, 0.0) / ser_n) / (skern[sdom] / 1e3) / 1e9 if skern[sdom] > 0 else 0.0
            iso = {"kernel": sdom, "kernel_ms_per_launch": round(skern[sdom], 4), "achieved": round(sach, 2),
                   "unit": "GB/s", "frac": round(sach / HBM_PEAK_GBS, 5), "batches": ser_n,
                   "stages_ms": {k: round(v, 4) for k, v in skern.items()},
                   "stages_alg_GBs": {k: round(ser_alg[k] / ser_n / (v / 1e3) / 1e9, 1)
                                      for k, v in skern.items() if ser_alg.get(k) and v > 0}}
        rk = iso["kernel"] if iso else dom  # the roofline kernel
        traffic, traffic_src, valu = None, None, None
        try:
            with open(a.pmc_json) as f:
                pmc = json.load(f)
            if pmc.get("config") == pmc_config_key(a) and rk in pmc.get("bytes_per_batch", {}):
                traffic = pmc["bytes_per_batch"][rk] * (B_ / pmc.get("images_per_batch", B_))
                traffic_src = f"{os.path.relpath(a.pmc_json)} ({pmc.get('correction', '')})"
            if pmc.get("config") == pmc_config_key(a):
                valu = {k: v * (B_ / pmc.get("images_per_batch", B_))
                        for k, v in pmc.get("valu_wave_insts_per_batch", {}).items()}
        except (OSError, ValueError):
            pass
        # measured device-to-device copy bandwidth (report the
        # roofline against it too): best of 3 copies of a 1 GiB buffer, bytes
        # read + written over the event time
        copy_gbs = None
        try:
            nbytes = 1 << 30
            xs = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
            ys = torch.empty_like(xs)
            best = None
            for _ in range(4):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                ys.copy_(xs)
                e1.record()
                e1.synchronize()
                t_ = e0.elapsed_time(e1) / 1e3
                best = t_ if best is None else min(best, t_)
            copy_gbs = round(2 * nbytes / best / 1e9, 1)
            del xs, ys
        except RuntimeError:
            pass
        result = {
            "metric": ("Mpixel/s device-resident PNG decode+bucket-resize (image + aligned mask pairs)" if png else
                       "Mpixel/s device-resident JPEG decode+bucket-resize at 1/2/4/8 MI355X"),
            "ms_per_step_per_rank": [round(t_ / a.steps * 1e3, 3) for t_ in per_rank_s],
            "value": round(px_all / dt_max / 1e6, 2),
            "windows": {"n": nwin, "steps_each": a.steps, "median_index": med,
                        "mpix_s": [round(v_, 2) for v_ in win_rate],
                        "spread_pct": round(100.0 * (max(win_rate) - min(win_rate)) / win_rate[med], 2),
                        "note": "value, ms_per_step and roofline_pipeline are the median window's (each window: "
                                "K steps between barriers + device syncs, max over ranks)"},
            "unit": "Mpixel/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(dt_max / a.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": (f"synthetic (seeded PIL PNG pool of {len(pool) // 2} RGB image + L8 mask pairs per rank, cycled)"
                     if png else f"synthetic ({a.shards} seeded WebDataset shards, {len(pool)} .jpg members on this "
                     f"rank, indexed in {wds_index_s * 1e3:.1f} ms by dg_wds_index, cycled)" if wds else
                     f"synthetic (seeded PIL JPEG pool of {a.pool} unique images, {len(pool)} of them resident "
                     f"on rank 0; {a.samples} logical samples, rank 0's slice [{lo}, {hi}))"),
            "config": {"workload": ("configs[2]: WebDataset shards (fake-imagenet-like {key}.jpg + {key}.cls, "
                                    f"W U[300,500] H U[250,500] q90), decode + bucket-resize to {a.size}/{a.ratio}")
                       if wds else ("configs[3]: file source sharded by rank/world_size "
                                    "(get_data_slice_multirank), 1M synthetic JPEGs (16,384-image pool, seed 4), "
                                    "decode + bucket-resize to 1024/32" if a.workload == "cfg4" else
                                    "configs[1]: file-source JPEGs, mixed aspect ratios, decode + bucket + "
                                    "crop/resize to 1024/32 buckets") if not png else
                                   (f"configs[4]{'' if a.encode else ' without re-encode'}: RGB PNG (PIL, zlib 6) "
                                    "+ L8 mask PNG pairs, mask aligned to the image's bucket, decode + crop/resize "
                                    f"to 1024/32{' + JPEG q92 re-encode of every payload' if a.encode else ''}"),
                       "decode_semantics": {"value": a.decode_semantics,
                                            "name": "zune-jpeg 0.5.12" if a.decode_semantics else "libjpeg-turbo",
                                            "note": "JPEG pixel stages (IDCT, upsampling, colour); 1 is the "
                                                    "reference's decoder and the mode INTEGRATION.md sets for the "
                                                    "drop-in (dg_image_config.decode_semantics)"},
                       "pre_encode_images": bool(a.encode),
                       "progressive_frac": a.progressive_frac, **({"ctx_opt": a.ctx_opt} if a.ctx_opt else {}),
                       "restart_marker_rows": a.rst_rows,
                       "images_per_step": B_, "pool": a.pool, "samples": a.samples,
                       "short_side": [a.short_min, a.short_max], "buckets": f"{a.size}/{a.ratio}/0.5/2.0",
                       "parallelism": f"dp{world} (sample shards, no collectives)"},
            # primary roofline: the dominant kernel's own duration -- HIP events on the slot stream around its
            # launches with the batch alone on the GPU (the serial batches after the timed region; rocprof's
            # per-dispatch average of the same kernels, profiles/, is the cross-check).  The span-based figure
            # over the overlapped timed region (roofline_overlapped_span) measures co-residency with the other
            # batches in flight, not the kernel.
            "roofline": ({"bound": "hbm", "kernel": iso["kernel"], "achieved": iso["achieved"], "peak": HBM_PEAK_GBS,
                          "unit": "GB/s", "frac": iso["frac"],
                          "traffic": round(traffic) if traffic else None, "traffic_source": traffic_src,
                          "alg_bytes_per_launch": round(ser_alg.get(iso["kernel"], 0.0) / ser_n),
                          "kernel_ms_per_launch": iso["kernel_ms_per_launch"],
                          "peak_measured_copy": copy_gbs,
                          "frac_of_measured_copy": round(iso["achieved"] / copy_gbs, 5) if copy_gbs else None,
                          "note": f"per launch = one {B_}-image batch; kernel time from HIP events with the batch "
                                  "alone on the GPU (roofline_isolated); kernel = the largest share of the timed "
                                  "region's stage spans (roofline_overlapped_span)"} if iso else
                         {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                          "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5),
                          "traffic": round(traffic) if traffic else None, "traffic_source": traffic_src,
                          "alg_bytes_per_launch": round(dom_alg), "kernel_ms_per_launch": round(dom_ms, 4),
                          "peak_measured_copy": copy_gbs,
                          "frac_of_measured_copy": round(achieved / copy_gbs, 5) if copy_gbs else None,
                          "note": "span-based (no serial batches run): HIP events over the overlapped timed region"}),
            "roofline_overlapped_span": {"kernel": dom, "achieved": round(achieved, 2), "frac": round(achieved / HBM_PEAK_GBS, 5),
                                         "kernel_span_ms_per_step": round(dom_ms, 4),
                                         "note": "HIP-event span of the kernel's launches on its slot stream over "
                                                 "the timed region, where consecutive batches overlap: co-residency, "
                                                 "not the kernel's own time"},
            "roofline_isolated": iso,
            # The pixel and entropy kernels are integer VALU / latency work, not HBM-bound: their VALU
            # issue rate (PMC SQ_INSTS_VALU per batch over the isolated kernel time) against the
            # MI355X peak of 256 CUs x 4 SIMDs x one wave-instruction per 2 cycles x 2.4 GHz.
            "roofline_valu": ({k: {"wave_insts": round(valu[k]),
                                   "achieved_T_per_s": round(valu[k] / (iso["stages_ms"][k] / 1e3) / 1e12, 4),
                                   "peak_T_per_s": VALU_PEAK_T,
                                   "frac": round(valu[k] / (iso["stages_ms"][k] / 1e3) / 1e12 / VALU_PEAK_T, 4)}
                               for k in valu if iso and iso["stages_ms"].get(k, 0) > 0.05}
                              if valu and iso else None),
            # SURVEY §8(d) B_alg of the whole path over the wall-clock step time
            "roofline_pipeline": {"alg_bytes_per_step": round(per_step_alg),
                                  "ms_per_step": round(dt_max / a.steps * 1e3, 4),
                                  "achieved_GBs": round(per_step_alg / (dt_max / a.steps) / 1e9, 2),
                                  "frac": round(per_step_alg / (dt_max / a.steps) / 1e9 / HBM_PEAK_GBS, 5),
                                  "frac_of_measured_copy": (round(per_step_alg / (dt_max / a.steps) / 1e9 / copy_gbs, 5)
                                                            if copy_gbs else None),
                                  "sum_of_stage_spans_ms": round(gpu_ms, 4)},
            "stages_ms_per_step": {k: round(v / steps, 4) for k, v in stage_tot.items()},
            "stages_alg_GBs": {k: round(stage_alg[k] / (stage_tot[k] / 1e3) / 1e9, 1)
                               for k in stage_tot if stage_alg.get(k) and stage_tot[k] > 0},
            "output_mpix_s": round(outpx_all / dt_max / 1e6, 2),
            "images_per_s": round(B_ * a.steps * world / dt_max, 1),
            "host_submit_ms_per_step": round(1e3 * host_s["submit"] / steps_all, 3),  # Python + dg_submit_device planning
            "host_submit_ms_per_step_per_rank": [round(1e3 * h_ / a.steps, 3) for h_ in per_rank_host],
            "host_submit_phases_ms_per_step": host_phases,
            "meta_bytes_per_batch": ctx.stat("meta_bytes"),
            "allocations": {k_: ctx.stat(k_) for k_ in ("allocs", "alloc_mb", "alloc_us", "reclaims", "retire_syncs",
                                                        "peak_device_mb", "max_device_mb", "budget_slots", "budget_splits",
                                                        "budget_frees", "budget_oom")},
            # per rank: wall ms per step in each dg_submit_device phase, the thread's CPU ms in the same
            # phases (wall >> cpu = blocking: allocation, driver locks, copies), and the slot wait
            "host_submit_phases_per_rank": [
                {"wall": {q: round(ph_all[r * len(HOST_PHASES) + j], 3) for j, q in
                          enumerate(HOST_PHASES)},
                 "cpu": {q: round(ph_all[len(HOST_PHASES) * world + r * (len(HOST_PHASES) - 1) + j], 3) for j, q in
                         enumerate(HOST_PHASES[:-1])}}
                for r in range(world)],
            "rank_cpus": (f"{len(pinned)} CPUs per rank, disjoint contiguous shares of the job's affinity set"
                          if pinned else "unpinned"),
            "e2e_host_mpix_s": round(e2e, 2) if e2e else None,
            "e2e_host_detail": ({"note": "host JPEG bytes in -> host RGB out, a dg_host_register'ed output pool "
                                         "reused, batches pipelined; outputs DMA'd from HBM into the pool",
                                 "outputs_direct_dma": e2e_direct, "output_GBs": round(e2e_out_gbs, 2),
                                 "d2h_pinned_GBs": round(d2h, 2) if d2h else None,
                                 "frac_of_d2h": round(e2e_out_gbs / d2h, 3) if d2h else None,
                                 "sync_fresh_arrays_mpix_s": round(e2e_sync, 2) if e2e_sync else None}
                                if e2e else None),
            "e2e_host_in_hbm_out_mpix_s": round(e2e_dev, 2) if e2e_dev else None,
            "e2e_decode_one": one,
            "corpus_gen_s": round(t_gen, 1),
            "corpus_generated_here": n_made if seq is not None else None,
            "stats": {"resync_rounds": ctx.stat("resync_rounds"), "fix_workgroups": ctx.stat("fix_workgroups"),
                      "write_mismatch": ctx.stat("write_mismatch"), "sync_iters_max": ctx.stat("sync_iters_max"),
                      "sub_bits": ctx.stat("sub_bits"), "lead_bits": a.lead_bits,
                      "png_chunks": ctx.stat("png_chunks"), "png_serial_fallbacks": ctx.stat("png_serial_fallbacks"),
                      "png_small_streams": ctx.stat("png_small_streams")},
            "wg_timing_us": ({f"{k}_{q}": ctx.stat(f"wg_{k}_{q}") / 1000 for k in ("sync", "write")
                              for q in ("span", "mean", "p90", "max")} if a.wg_timing else None),
        }
        if world == 1 and not a.no_cpu_baseline:
            result["cpu_baseline"] = cpu_baseline(pool, targets, a.cpu_seconds, a.encode, a.decode_semantics)
            result["cpu_baseline_pillow"] = pillow_baseline(pool, targets, a.cpu_seconds, a.encode)
        else:
            result["cpu_baseline"] = None
        if png or wds:  # the PMC file is for the configs[1] workload
            result["roofline"]["traffic"] = None
            result["roofline"]["traffic_source"] = None
        line = json.dumps(result)
        print(line, flush=True)
        if a.out:
            with open(a.out, "w") as f:
                f.write(line + "\n")
    ctx.free(d_arena)
    for p_ in d_out:
        ctx.free(p_)
    ctx.close()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return 0


def close_contexts() -> None:
    """Every dg_ctx this process opened, also when main() raised (VERDICT r4:
    process exit with live contexts).  The launcher parent never loads the library."""
    L = sys.modules.get("datago_amd._lib")
    if L is not None:
        L.close_all()


if __name__ == "__main__":
    try:
        rc = main()
    finally:
        close_contexts()
    sys.exit(rc)
