"""Per-kernel duration summary from a rocprofv3 SQLite (rocpd) results file:
python tools/rocpd_stats.py run_results.db [--csv out.csv]"""
import argparse
import collections
import sqlite3

ap = argparse.ArgumentParser()
ap.add_argument("db")
ap.add_argument("--csv")
a = ap.parse_args()
c = sqlite3.connect(a.db)
rows = list(c.execute('select name, start, "end", grid_x, workgroup_x, lds_size, scratch_size, vgpr_count '
                      'from kernels order by start'))
agg = collections.defaultdict(list)
for r in rows:
    agg[r[0].split("(")[0]].append(((r[2] - r[1]) / 1e6,) + tuple(r[3:]))
lines = ["kernel,calls,total_ms,avg_ms,max_ms,grid,wg,lds,scratch,vgpr"]
for k, v in sorted(agg.items(), key=lambda kv: -sum(x[0] for x in kv[1])):
    ds = [x[0] for x in v]
    lines.append(f"{k},{len(v)},{sum(ds):.3f},{sum(ds) / len(ds):.4f},{max(ds):.3f},{v[0][1]},{v[0][2]},{v[0][3]},"
                 f"{v[0][4]},{v[0][5]}")
print("\n".join(lines))
if a.csv:
    open(a.csv, "w").write("\n".join(lines) + "\n")
