"""Per-stage spans of the last N batches of a rocprofv3 kernel trace (rocpd
SQLite): bench.py ends with batches run one at a time (its isolated pass,
`roofline_isolated`), so their stage spans -- first kernel start to last
kernel end of the stage, the same bracket as bench.py's HIP events -- are the
rocprof figures the bench line's `kernel_ms_per_launch` must agree with.

    python tools/rocpd_stages.py run_results.db [--batches 3]

Stages follow tools/pmc_traffic.py's mapping: k_resize_hb/k_resize_h launches
before a batch's first k_resize_v are call 1's H pass (resize_h1)."""
import argparse
import collections
import sqlite3


def stage_of(name, state):
    n = name.split("(")[0].replace("void ", "").replace("dg::", "").split("<")[0]
    if n.startswith("k_destuff"):
        return "destuff"
    if n.startswith("k_huff_sync"):
        state["nv"] = 0
        return "huff_sync"
    if n.startswith("k_huff_"):
        return n[2:]
    if n.startswith("k_resize_v"):
        state["nv"] += 1
        return "resize_v1" if state["nv"] == 1 else "resize_v2"
    if n.startswith("k_resize_h"):
        return "resize_h1" if state["nv"] == 0 else "resize_h2"
    if n.startswith("k_idct"):
        return "idct"
    return n[2:] if n.startswith("k_") else n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--batches", type=int, default=3)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    ks = sorted((r[1], r[2], r[0]) for r in c.execute('select name, start, "end" from kernels') if "dg::" in r[0])
    starts = [i for i, (_, _, n) in enumerate(ks) if "k_huff_sync" in n]
    if len(starts) < a.batches:
        raise SystemExit("not enough batches in the trace")
    first = starts[-a.batches]
    spans = collections.defaultdict(list)
    state = {"nv": 0}
    batch = -1
    cur = {}
    for s, e, n in ks[first:]:
        if "k_huff_sync" in n:
            if cur:
                for k, (b0, b1, cnt) in cur.items():
                    spans[k].append(((b1 - b0) / 1e6, cnt))
            cur = {}
            batch += 1
        st = stage_of(n, state)
        b0, b1, cnt = cur.get(st, (s, e, 0))
        cur[st] = (min(b0, s), max(b1, e), cnt + 1)
    for k, (b0, b1, cnt) in cur.items():
        spans[k].append(((b1 - b0) / 1e6, cnt))
    print(f"stage spans of the last {a.batches} batches (ms per batch: mean, per batch; kernel launches per batch)")
    for k, v in sorted(spans.items(), key=lambda kv: -sum(x for x, _ in kv[1])):
        ms = [x for x, _ in v]
        print(f"{k},{sum(ms) / len(ms):.3f},{' '.join(f'{x:.3f}' for x in ms)},{v[0][1]}")


if __name__ == "__main__":
    main()
