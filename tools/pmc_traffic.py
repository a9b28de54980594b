"""Per-stage HBM traffic of bench.py from rocprofv3 PMC passes
(tools/gpu_pmc.sh: separate FETCH_SIZE and WRITE_SIZE passes).

Kernels are mapped to bench stages by dispatch order within each batch
(k_huff_sync starts a batch; k_resize_hb launches before a batch's first
k_resize_v are call 1's H pass, later ones call 2's; the first k_resize_v is
call 1's V pass, the second call 2's).  FETCH_SIZE is in KiB and, on gfx950,
reports half the bytes of wide (16 B/lane) coalesced reads
(MI355X_MICROARCH.md, HBM section): it is doubled here and labelled so;
WRITE_SIZE is taken as is.  Output: JSON with bytes per batch per stage.

  python tools/pmc_traffic.py gpurun_out/pmc > profiles/r01/pmc_traffic.json
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def stage_sequence(rows):
    """[(dispatch_id, stage)] for the dg:: kernels, in dispatch order."""
    out = []
    phase = None
    nv = 0
    for r in sorted(rows, key=lambda r: int(r["Dispatch_Id"])):
        k = r["Kernel_Name"]
        if "dg::" not in k:
            continue
        name = k.split("(")[0].replace("void ", "").replace("dg::", "").split("<")[0]
        if name.startswith("k_huff_sync"):
            nv = 0
            phase = "h1"
        if name.startswith("k_destuff"):
            st = "destuff"
        elif name.startswith("k_huff_"):
            st = name[2:].replace("huff_", "huff_")
        elif name.startswith("k_resize_v"):
            nv += 1
            st = "resize_v1" if nv == 1 else "resize_v2"
            phase = "h2"
        elif name.startswith("k_resize_h"):
            st = "resize_h1" if phase in (None, "h1") else "resize_h2"
        elif name.startswith("k_idct"):
            st = "idct"  # k_idct, k_idct_t (one lane per block)
        else:
            st = name[2:]  # color, coeffs, copy
        out.append((int(r["Dispatch_Id"]), st))
    return out


def main(root, config=None, images_per_batch=None):
    res = {}
    for counter, sub in (("FETCH_SIZE", "fetch"), ("WRITE_SIZE", "write")):
        files = glob.glob(os.path.join(root, sub, "**", "*counter_collection.csv"), recursive=True)
        rows = [r for f in files for r in csv.DictReader(open(f)) if r["Counter_Name"] == counter]
        seq = dict(stage_sequence(rows))
        per = defaultdict(float)
        nbatch = sum(1 for r in rows if "k_huff_sync" in r["Kernel_Name"])
        for r in rows:
            d = int(r["Dispatch_Id"])
            if d in seq:
                per[seq[d]] += float(r["Counter_Value"]) * 1024.0
        res[counter] = ({k: v / max(nbatch, 1) for k, v in per.items()}, nbatch)
    # VALU wave-instructions per stage (the "sq" pass), for the compute-side roofline
    files = glob.glob(os.path.join(root, "sq", "**", "*counter_collection.csv"), recursive=True)
    rows = [r for f in files for r in csv.DictReader(open(f)) if r["Counter_Name"] == "SQ_INSTS_VALU"]
    valu = defaultdict(float)
    if rows:
        seq = dict(stage_sequence(rows))
        nbv = sum(1 for r in rows if "k_huff_sync" in r["Kernel_Name"])
        for r in rows:
            d = int(r["Dispatch_Id"])
            if d in seq:
                valu[seq[d]] += float(r["Counter_Value"])
        valu = {k: v / max(nbv, 1) for k, v in valu.items()}
    fetch, nb = res["FETCH_SIZE"]
    write, _ = res["WRITE_SIZE"]
    # request-size passes (tools/gpu_calib.sh calibrated them against known byte counts):
    # read bytes = 32 n32 + 64 n64 + 128 n128, write bytes = 32 (n - n64) + 64 n64
    def per_stage(sub, weights):
        files = glob.glob(os.path.join(root, sub, "**", "*counter_collection.csv"), recursive=True)
        rows = [r for f in files for r in csv.DictReader(open(f)) if r["Counter_Name"] in weights]
        if not rows:
            return None
        first = next(iter(weights))  # one row per dispatch for the stage sequence (it counts launches)
        seq = dict(stage_sequence([r for r in rows if r["Counter_Name"] == first]))
        nbq = len({int(r["Dispatch_Id"]) for r in rows if "k_huff_sync" in r["Kernel_Name"]})
        acc = defaultdict(float)
        for r in rows:
            d = int(r["Dispatch_Id"])
            if d in seq:
                acc[seq[d]] += weights[r["Counter_Name"]] * float(r["Counter_Value"])
        return {k: v / max(nbq, 1) for k, v in acc.items()}
    rd_req = per_stage("req", {"TCC_EA0_RDREQ_32B_sum": 32.0, "TCC_EA0_RDREQ_64B_sum": 64.0,
                               "TCC_EA0_RDREQ_128B_sum": 128.0})
    wr_req = per_stage("wreq", {"TCC_EA0_WRREQ_sum": 32.0, "TCC_EA0_WRREQ_64B_sum": 32.0})
    stages = sorted(set(fetch) | set(write))
    out = {
        "config": config,
        "images_per_batch": int(images_per_batch) if images_per_batch else None,
        "source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of bench.py (tools/gpu_pmc.sh)",
        "batches": nb,
        "correction": ("reads: request-size counters (32 n32 + 64 n64 + 128 n128), writes: WRITE_SIZE; "
                       "calibrated on known bytes (profiles/r06/calib/fetch_calib.json: FETCH_SIZE x2 = the bytes "
                       "for 4/8/16-B and partial-line 16-B reads; a partial 128-B line is fetched whole)"
                       if rd_req else "FETCH_SIZE x2 (calibrated: profiles/r06/calib/fetch_calib.json)"),
        "bytes_per_batch": {s: round((rd_req.get(s, 0.0) if rd_req else 2.0 * fetch.get(s, 0.0)) + write.get(s, 0.0))
                            for s in stages},
        "read_bytes_by_request_size": {s: round(v) for s, v in sorted(rd_req.items())} if rd_req else None,
        "write_bytes_by_request_size": {s: round(v) for s, v in sorted(wr_req.items())} if wr_req else None,
        "fetch_bytes_per_batch_x2": {s: round(2.0 * fetch.get(s, 0.0)) for s in stages},
        "write_bytes_per_batch": {s: round(write.get(s, 0.0)) for s in stages},
        "valu_wave_insts_per_batch": {s: round(v) for s, v in sorted(valu.items())},
    }
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    # usage: pmc_traffic.py ROOT CONFIG_KEY IMAGES_PER_BATCH  (CONFIG_KEY as bench.pmc_config_key)
    main(*(sys.argv[1:4] if len(sys.argv) > 1 else ["gpurun_out/pmc"]))
