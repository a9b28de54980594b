"""Debug probe: which entropy workgroups are the long pole of k_huff_sync /
k_huff_write?  Decodes configs[1]-distribution batches one at a time with
per-workgroup timestamps (option wg_timing, dump via DG_WG_DUMP) and prints
the slowest workgroups with their image's coded density.

    python tools/probe/wg_probe.py [--batches 2] [--opt key=value ...]
"""
import argparse
import os
import sys
import tempfile

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", type=int, default=2)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--opt", action="append", default=[])
    ap.add_argument("--top", type=int, default=12)
    a = ap.parse_args()
    from datago_amd import synth
    from datago_amd import _lib as L
    n = a.batches * a.batch
    idx = list(range(n))
    synth.generate_pool_images(2, 4096, idx, 16, 256, 2048, 0.0)
    pool = synth.load_pool_images(2, 4096, idx, 256, 2048, 0.0)
    dump = os.path.join(tempfile.mkdtemp(), "wg.txt")
    os.environ["DG_WG_DUMP"] = dump
    ctx = L.Context(0, crop_and_resize=True, default_image_size=1024, downsampling_ratio=32, min_aspect_ratio=0.5,
                    max_aspect_ratio=2.0)
    ctx.set_option("wg_timing", 1)
    for kv in a.opt:
        k, v = kv.split("=")
        ctx.set_option(k, int(v))
    ctx.decode_batch(pool[:a.batch])  # warm-up (not dumped)
    os.remove(dump) if os.path.exists(dump) else None
    for b in range(a.batches):
        res = ctx.decode_batch(pool[b * a.batch:(b + 1) * a.batch])
        assert all(r[0] == 0 for r in res)
    recs, cur = [], []
    for line in open(dump):
        if line.startswith("end"):
            recs.append(cur)
            cur = []
        else:
            cur.append([int(x) for x in line.split()])
    for bi, rs in enumerate(recs):
        for kern, name in ((0, "sync"), (1, "write")):
            r = [x for x in rs if x[0] == kern]
            if not r:
                continue
            t0 = min(x[4] for x in r)
            span = (max(x[5] for x in r) - t0) / 100.0
            durs = sorted(((x[5] - x[4]) / 100.0, x) for x in r)
            mean = sum(d for d, _ in durs) / len(durs)
            print(f"batch {bi} {name}: {len(r)} wgs span {span:.0f} us mean {mean:.0f} us")
            for d, x in durs[::-1][:a.top]:
                _, _, img, item0, s, e, scan_len, blocks, sub_bits, nsub, lead, px = x
                print(f"   {d:7.0f} us start {(s - t0) / 100:6.0f} img {img:3d} item0 {item0:5d} nsub {nsub:4d} "
                      f"sub_bits {sub_bits:5d} lead {lead:5d} bits/blk {8 * scan_len / blocks:6.1f} "
                      f"scan {scan_len >> 10} KiB px {px / 1e6:.2f} M")
            # mean workgroup time by coded bits per block (and lead-in)
            bins = {}
            for d, x in durs:
                bpb = 8 * x[6] / x[7]
                key = (x[10], min(int(bpb // 20) * 20, 200))
                bins.setdefault(key, []).append(d)
            print("   by (lead, bits/blk bin):", " ".join(
                f"{k[0]}/{k[1]}:{sum(v) / len(v):.0f}x{len(v)}" for k, v in sorted(bins.items())))
            # images by total workgroup time
            late = sorted(((x[5] - t0) / 100.0, x) for x in r)[::-1][:5]
            print("   last to finish:", [(round(t), x[2], x[3]) for t, x in late])


if __name__ == "__main__":
    main()
