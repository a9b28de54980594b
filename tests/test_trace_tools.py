"""The rocprof trace summaries behind the round-4 evidence (tools/rocpd_stages.py:
isolated stage spans that bench.py's roofline must agree with;
tools/trace_window.py: GPU busy fraction and idle gaps) on a synthetic rocpd
database with known answers."""
import os
import sqlite3
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _db(path):
    c = sqlite3.connect(path)
    c.execute('create table kernels (name text, start integer, "end" integer, grid_x integer, workgroup_x integer, '
              'lds_size integer, scratch_size integer, vgpr_count integer)')
    t = 0
    rows = []
    for b in range(4):  # four batches run one at a time: sync, write, idct, 2 H launches, V, H2, V2
        for name, ms in (("dg::k_huff_sync<false>", 1.0), ("dg::k_huff_write", 0.5), ("dg::k_idct_t", 0.4),
                         ("void dg::k_resize_hb<16, true, true>", 0.7), ("void dg::k_resize_hb<8, true, true>", 0.3),
                         ("dg::k_resize_v", 0.6), ("void dg::k_resize_hb<8, false, false>", 0.1),
                         ("dg::k_resize_v", 0.05)):
            rows.append((name + "(args)", t, t + int(ms * 1e6), 1, 256, 0, 0, 32))
            t += int(ms * 1e6) + 100_000  # 0.1 ms idle between kernels
    c.executemany("insert into kernels values (?,?,?,?,?,?,?,?)", rows)
    c.commit()
    c.close()
    return t


def test_rocpd_stages_isolated_spans(tmp_path):
    db = str(tmp_path / "run_results.db")
    _db(db)
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "rocpd_stages.py"), db, "--batches", "3"],
                         capture_output=True, text=True, check=True).stdout
    spans = {l.split(",")[0]: l.split(",") for l in out.strip().splitlines()[1:]}
    # resize_h1 = the two H launches before the first V: 0.7 + 0.1 idle + 0.3 ms
    assert abs(float(spans["resize_h1"][1]) - 1.1) < 1e-6 and spans["resize_h1"][3] == "2"
    assert abs(float(spans["huff_sync"][1]) - 1.0) < 1e-6
    assert abs(float(spans["resize_v1"][1]) - 0.6) < 1e-6 and abs(float(spans["resize_v2"][1]) - 0.05) < 1e-6
    assert abs(float(spans["resize_h2"][1]) - 0.1) < 1e-6


def test_trace_window_busy_fraction(tmp_path):
    db = str(tmp_path / "run_results.db")
    _db(db)
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "trace_window.py"), db],
                         capture_output=True, text=True, check=True).stdout
    first = out.splitlines()[0]
    # 4 batches x (3.65 ms of kernels + 8 x 0.1 ms gaps), less the gap after the last kernel: 14.6 / 17.7 ms
    busy = float(first.split("kernels busy ")[1].split("%")[0])
    assert first.startswith("window 17.70 ms") and abs(busy - 100 * 14.6 / 17.7) < 0.1, first
    assert "idle gaps: 31" in out
