"""Instructions per Huffman symbol of the GPU entropy kernels (VERDICT r1
item 5): PMC wave-instruction counts per batch (profiles/r02/pmc_traffic.json
VALU, v2_pmc_summary.txt SALU) over the symbols of the same batches, counted
by the oracle's decoder (test infrastructure, run on the CPU).

    python tools/entropy_per_symbol.py [--batches 3] [--out profiles/r02/entropy_per_symbol.json]

Counts: a wave instruction serves 64 lanes, each decoding its own symbol, so
per-lane instructions per symbol = wave instructions x 64 / symbols decoded.
k_huff_sync decodes every symbol of its range plus a lead-in (6144 bits for
6-block MCUs, 2048 otherwise) and any re-decodes; the figures below divide by
the stream's symbols (what the pipeline must decode once), so they include
that redundancy; k_huff_write decodes each symbol once."""
import argparse
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", type=int, default=3)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--pool", type=int, default=4096)
    ap.add_argument("--pmc", default=os.path.join(ROOT, "profiles/r02/pmc_traffic.json"))
    ap.add_argument("--summary", default=os.path.join(ROOT, "profiles/r02/v2_pmc_summary.txt"))
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles/r02/entropy_per_symbol.json"))
    ap.add_argument("--workers", type=int, default=8)
    a = ap.parse_args()
    from datago_amd import synth
    from oracle import oracle as O
    idx = list(range(a.batches * a.batch))
    synth.generate_pool_images(2, a.pool, idx, workers=a.workers)
    imgs = synth.load_pool_images(2, a.pool, idx)
    L = O.lib()
    L.oj_reset_symbol_count()
    coded = 0
    for d in imgs:
        st, _ = O.jpeg_decode(d)
        assert st == 0
        coded += len(d)
    symbols = L.oj_symbol_count() / a.batches
    pmc = json.load(open(a.pmc))
    valu = pmc["valu_wave_insts_per_batch"]
    salu = {}
    cur = None
    for line in open(a.summary):
        m = re.match(r"^(\S.*)$", line.rstrip())
        if m and not line.startswith(" "):
            cur = m.group(1)
        m = re.match(r"^\s+SQ_INSTS_SALU\s+([\d,\.]+)", line)
        if m and cur:
            key = "huff_sync" if "k_huff_sync" in cur else "huff_write" if "k_huff_write" in cur else None
            if key:
                salu[key] = float(m.group(1).replace(",", ""))
    out = {"symbols_per_batch": symbols, "coded_bytes_per_batch": coded / a.batches,
           "sample": f"pool images 0..{len(idx) - 1} (seed 2, the bench's first {a.batches} batches of {a.batch})",
           "per_symbol": {}}
    for k in ("huff_sync", "huff_write"):
        out["per_symbol"][k] = {"valu_lane_insts": valu[k] * 64 / symbols,
                                "salu_insts_per_wave_symbol": salu.get(k, float("nan")) * 64 / symbols,
                                "valu_wave_insts_per_batch": valu[k], "salu_insts_per_batch": salu.get(k)}
    json.dump(out, open(a.out, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
