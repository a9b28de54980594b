"""Latency chain of dg_decode_one's coalesced batches from a rocprofv3 trace
(rocpd SQLite): the last `--batches` batches of the run (a batch starts at a
k_destuff_count), per batch the span from its first to its last kernel, the
kernels on that chain with their start offsets, and the gaps between them.

    python tools/one_chain.py run_results.db [--batches 200]"""
import argparse
import collections
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--batches", type=int, default=200)
    ap.add_argument("--timeline", type=float, default=0.0, help="print every kernel within this many us of a mid batch")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = [(r[0].split("(")[0].replace("void ", "").replace("dg::", ""), r[1], r[2], r[3], r[4])
            for r in c.execute('select name, start, "end", grid_x, stream_id from kernels order by start')]
    # batches: a stream's kernels from one k_destuff_count to the next
    per_stream = collections.defaultdict(list)
    for n, s, e, g, st in rows:
        per_stream[st].append((n, s, e, g, st))
    batches = []
    for st, ks in per_stream.items():
        cur = None
        for k in ks:
            # a batch starts at its descriptor pull (or, without one, its first destuff)
            starts = k[0].startswith("k_meta_pull") or (k[0].startswith("k_destuff_count") and not (
                cur and cur[-1][0].startswith("k_meta_pull")))
            if starts:
                if cur:
                    batches.append(cur)
                cur = [k]
            elif cur is not None:
                cur.append(k)
        if cur:
            batches.append(cur)
    batches.sort(key=lambda b: b[0][1])
    batches = [b for b in batches if max(k[3] for k in b) < 2_000_000][-a.batches:]  # small (coalesced) batches
    spans = sorted((b[-1][2] - b[0][1]) / 1e3 for b in batches)
    if not spans:
        print("no batches")
        return
    print(f"{len(batches)} batches: span p50 {spans[len(spans) // 2]:.0f} us, p90 {spans[int(0.9 * len(spans))]:.0f} us")
    agg = collections.defaultdict(lambda: [0, 0.0, 0.0])
    for b in batches:
        t0 = b[0][1]
        for n, s, e, g, _ in b:
            x = agg[n.split("<")[0]]
            x[0] += 1
            x[1] += (e - s) / 1e3
            x[2] += (s - t0) / 1e3
    print("kernel,launches_per_batch,avg_us,avg_start_offset_us")
    for n, (k, d, o) in sorted(agg.items(), key=lambda kv: kv[1][2] / kv[1][0]):
        print(f"{n},{k / len(batches):.2f},{d / k:.1f},{o / k:.0f}")
    if a.timeline:
        t_sel = batches[len(batches) // 2][0][1]
        print(f"timeline around t={t_sel} (all streams, {a.timeline} us):")
        for n, s, e, g, st in rows:
            if t_sel <= s <= t_sel + a.timeline * 1e3:
                print(f"  {(s - t_sel) / 1e3:8.1f} {(e - t_sel) / 1e3:8.1f} s{st} {n[:40]} grid={g}")


if __name__ == "__main__":
    main()
