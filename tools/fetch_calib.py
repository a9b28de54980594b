"""FETCH_SIZE / WRITE_SIZE correction factors per access shape on gfx950
(VERDICT r5 item 1), from tools/fetch_calib's known-byte dispatches and two
rocprofv3 --pmc passes over it (tools/gpu_calib.sh).

    python tools/fetch_calib.py OUT > profiles/r06/calib/fetch_calib.json

OUT holds fetch.jsonl / write.jsonl (the program's per-dispatch lines, one
run per pass) and fetch/ write/ (the passes' counter_collection.csv).  For
each shape: counter bytes (FETCH_SIZE and WRITE_SIZE are in KiB), the bytes
the kernel moved, and factor = moved / counted (multiply a counter reading of
that shape by it).  Dispatches are matched by order (the helper fills the
program makes through the runtime are skipped by name)."""
import csv
import glob
import json
import os
import sys


def _rows(root, sub, counter):
    files = glob.glob(os.path.join(root, sub, "**", "*counter_collection.csv"), recursive=True)
    rows = [r for f in files for r in csv.DictReader(open(f)) if r["Counter_Name"] == counter]
    rows = [r for r in rows if not r["Kernel_Name"].startswith("__amd")]
    by = {}
    for r in rows:  # one row per dispatch (summed over dimensions if split)
        d = int(r["Dispatch_Id"])
        by[d] = by.get(d, 0.0) + float(r["Counter_Value"])
    return [by[d] for d in sorted(by)], [r["Kernel_Name"] for r in sorted(rows, key=lambda r: int(r["Dispatch_Id"]))]


def main(root):
    out = {"source": "tools/fetch_calib.hip dispatches over a 2 GiB buffer (past the 256 MiB Infinity Cache), "
                     "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes (tools/gpu_calib.sh)",
           "shapes": {}}
    for sub, counter in (("fetch", "FETCH_SIZE"), ("write", "WRITE_SIZE")):
        lines = [json.loads(x) for x in open(os.path.join(root, sub + ".jsonl")) if x.startswith("{")]
        vals, names = _rows(root, sub, counter)
        if len(vals) != len(lines):
            raise SystemExit(f"{sub}: {len(vals)} PMC dispatches vs {len(lines)} program lines")
        for ln, v in zip(lines, vals):
            if ln["rep"] != 1:
                continue
            cb = v * 1024.0
            s = out["shapes"].setdefault(ln["kernel"], {"dir": ln["dir"], "bytes": ln["bytes"]})
            s[counter] = round(cb)
            if (ln["dir"] == "read") == (counter == "FETCH_SIZE"):
                s["factor"] = round(ln["bytes"] / cb, 4) if cb else None
                s["GBs"] = ln["GBs"]
    # request-size passes: bytes = 32 n32 + 64 n64 + 128 n128 (reads), 32 (n - n64) + 64 n64 (writes)
    for sub, ctrs in (("req", ("TCC_EA0_RDREQ_sum", "TCC_EA0_RDREQ_32B_sum", "TCC_EA0_RDREQ_64B_sum",
                                "TCC_EA0_RDREQ_128B_sum")),
                      ("wreq", ("TCC_EA0_WRREQ_sum", "TCC_EA0_WRREQ_64B_sum"))):
        path = os.path.join(root, sub + ".jsonl")
        if not os.path.exists(path):
            continue
        lines = [json.loads(x) for x in open(path) if x.startswith("{")]
        cols = {c: _rows(root, sub, c)[0] for c in ctrs}
        if any(len(v) != len(lines) for v in cols.values()):
            raise SystemExit(f"{sub}: dispatch count mismatch")
        for j, ln in enumerate(lines):
            if ln["rep"] != 1:
                continue
            s = out["shapes"][ln["kernel"]]
            v = {c: cols[c][j] for c in ctrs}
            if sub == "req":
                s["rdreq"] = {"all": round(v[ctrs[0]]), "32B": round(v[ctrs[1]]), "64B": round(v[ctrs[2]]),
                              "128B": round(v[ctrs[3]])}
                rb = 32 * v[ctrs[1]] + 64 * v[ctrs[2]] + 128 * v[ctrs[3]]
                s["read_bytes_by_request_size"] = round(rb)
                if ln["dir"] == "read":
                    s["factor_by_request_size"] = round(ln["bytes"] / rb, 4) if rb else None
            else:
                s["wrreq"] = {"all": round(v[ctrs[0]]), "64B": round(v[ctrs[1]])}
                wb = 32 * (v[ctrs[0]] - v[ctrs[1]]) + 64 * v[ctrs[1]]
                s["write_bytes_by_request_size"] = round(wb)
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/calib")
