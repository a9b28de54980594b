"""GPU timeline over a window of a rocprofv3 SQLite (rocpd) trace: how busy the
kernels and the copy engines were, per-kernel totals and the idle gaps.  For
legs that are latency- rather than throughput-bound (dg_decode_one).

    python tools/trace_window.py run_results.db [--last-s 0.5] [--first-s 0]

--last-s W: the last W seconds of the trace (the decode_one leg runs last in
bench.py); 0 = the whole trace."""
import argparse
import collections
import sqlite3


def cols(c, name):
    return [r[1] for r in c.execute(f"pragma table_info('{name}')")]


def union(iv):
    tot, cur_s, cur_e = 0, None, None
    for s, e in sorted(iv):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def gaps(iv, t0, t1):
    out, last = [], t0
    for s, e in sorted(iv):
        if s > last:
            out.append(s - last)
        last = max(last, e)
    if t1 > last:
        out.append(t1 - last)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--last-s", type=float, default=0.0)
    ap.add_argument("--first-s", type=float, default=0.0)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    names = {r[0] for r in c.execute("select name from sqlite_master where type in ('table', 'view')")}
    ks = [(r[0].split("(")[0], r[1], r[2]) for r in c.execute('select name, start, "end" from kernels')]
    cps = []
    if "memory_copies" in names:
        cc = cols(c, "memory_copies")
        size_col = next((x for x in ("size", "bytes", "copy_bytes") if x in cc), None)
        kind_col = next((x for x in ("name", "operation", "kind", "direction") if x in cc), None)
        q = f'select start, "end", {size_col or 0}, {kind_col or "0"} from memory_copies'
        cps = [(r[0], r[1], r[2] or 0, str(r[3])) for r in c.execute(q)]
    t_end = max([e for _, _, e in ks] + [e for _, e, _, _ in cps])
    t_beg = min([s for _, s, _ in ks] + [s for s, _, _, _ in cps])
    w0 = t_end - int(a.last_s * 1e9) if a.last_s > 0 else t_beg
    w1 = t_end
    if a.first_s > 0:
        w0, w1 = t_beg, t_beg + int(a.first_s * 1e9)
    ks = [(n, max(s, w0), min(e, w1)) for n, s, e in ks if e > w0 and s < w1]
    cps = [(max(s, w0), min(e, w1), b, k) for s, e, b, k in cps if e > w0 and s < w1]
    W = w1 - w0
    kb = union([(s, e) for _, s, e in ks])
    cb = union([(s, e) for s, e, _, _ in cps])
    ab = union([(s, e) for _, s, e in ks] + [(s, e) for s, e, _, _ in cps])
    print(f"window {W / 1e6:.2f} ms: kernels busy {kb / W:.1%}, copies busy {cb / W:.1%}, any {ab / W:.1%}")
    g = sorted(gaps([(s, e) for _, s, e in ks] + [(s, e) for s, e, _, _ in cps], w0, w1))
    if g:
        print(f"idle gaps: {len(g)}, total {sum(g) / 1e6:.2f} ms, median {g[len(g) // 2] / 1e3:.1f} us, "
              f"p90 {g[int(len(g) * 0.9)] / 1e3:.1f} us, max {g[-1] / 1e3:.1f} us")
    per = collections.defaultdict(lambda: [0, 0])
    for n, s, e in ks:
        per[n][0] += 1
        per[n][1] += e - s
    print("kernel,calls,total_ms,avg_us,share_of_window")
    for n, (k, t) in sorted(per.items(), key=lambda kv: -kv[1][1])[:25]:
        print(f"{n},{k},{t / 1e6:.2f},{t / k / 1e3:.1f},{t / W:.1%}")
    byk = collections.defaultdict(lambda: [0, 0, 0])
    for s, e, b, k in cps:
        byk[k][0] += 1
        byk[k][1] += e - s
        byk[k][2] += b
    for k, (n, t, b) in byk.items():
        print(f"copies {k}: {n}, {t / 1e6:.2f} ms busy, {b / 1e6:.1f} MB, {b / max(t, 1):.2f} GB/s while busy, "
              f"mean {b / max(n, 1) / 1e3:.0f} KB")


if __name__ == "__main__":
    main()
