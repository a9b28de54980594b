"""Summarise rocprofv3 --pmc passes (tools/gpu_pmc.sh): per kernel, the mean
per dispatch of every counter collected, plus derived ratios."""
import csv
import glob
import os
import sys
from collections import defaultdict


def load(root):
    per = defaultdict(lambda: defaultdict(list))  # kernel -> counter -> values per dispatch
    for f in glob.glob(os.path.join(root, "*", "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                k = r.get("Kernel_Name", r.get("Kernel-Name", "?"))
                k = k.split("(")[0].replace("void ", "")
                per[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return per


def main(root="gpurun_out/pmc"):
    per = load(root)
    rows = []
    for k, cs in per.items():
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        rows.append((k, m))
    rows.sort(key=lambda x: -x[1].get("SQ_WAVE_CYCLES", 0))
    for k, m in rows:
        d = dict(m)
        if "FETCH_SIZE" in d:
            d["FETCH_MB_x2"] = d["FETCH_SIZE"] * 2 / 1024  # gfx950: FETCH_SIZE (KB) reports 1/2 of wide reads
        if "WRITE_SIZE" in d:
            d["WRITE_MB"] = d["WRITE_SIZE"] / 1024
        wc = d.get("SQ_WAVE_CYCLES")
        if wc:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                if c in d:
                    d[c + "_frac"] = d[c] / wc
        if d.get("SQ_WAVES"):
            for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS"):
                if c in d:
                    d[c + "_per_wave"] = d[c] / d["SQ_WAVES"]
        print(k)
        for c in sorted(d):
            print(f"   {c:28s} {d[c]:,.3f}")


if __name__ == "__main__":
    main(*sys.argv[1:])
