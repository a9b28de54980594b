"""Per-scan timing of k_prog_scan (debug): the configs[1] pool's largest
progressive file alone, then a 64-image slice of the pool, for each value of
option prog_chain.  Writes DG_PROG_DUMP lines (scan, image, ns, comp, ss, se,
ah, al, len, level, pflags, t0, t1 [10 ns ticks], blocks, pixels) under
gpurun_out/prog3/ and prints each batch's wall time and stage times."""
import os
import sys
import time

sys.path.insert(0, ".")
from datago_amd import synth  # noqa: E402
from datago_amd import _lib as L  # noqa: E402

OUT = os.environ.get("OUT", "gpurun_out/prog3")


def main():
    os.makedirs(OUT, exist_ok=True)
    spec = synth.mixed_spec(2, 256, 256, 2048)
    order = sorted(range(256), key=lambda i: -spec[i][0] * spec[i][1])
    def mk(i):
        w, h, q, ss, g = spec[i]
        return synth.make_jpeg(2 * 1_000_003 + i, w, h, q, ss, g, 0, progressive=True)
    big = [mk(order[0])]
    t = time.time()
    pool = [mk(i) for i in range(64)]
    print("generated", len(pool), "in", round(time.time() - t, 1), "s", flush=True)
    for chain in [int(x) for x in os.environ.get("CHAINS", "0,100").split(",")]:
        ctx = L.Context(0, crop_and_resize=True, default_image_size=1024, downsampling_ratio=32,
                        min_aspect_ratio=0.5, max_aspect_ratio=2.0)
        ctx.set_option("progressive", 1)
        ctx.set_option("prog_chain", chain)
        for name, batch in (("largest", big), ("pool64", pool)):
            for rep in range(2):
                ctx.set_option("timing", 1)
                ctx.set_option("wg_timing", 1 if rep else 0)
                os.environ["DG_PROG_DUMP"] = f"{OUT}/dump_{name}_c{chain}.txt" if rep else ""
                t = time.perf_counter()
                res = ctx.decode_batch(batch)
                dt = time.perf_counter() - t
                bad = [r[0] for r in res if r[0] != 0]
                tm = ctx.timings()
                print(f"chain {chain} {name} rep {rep} wall {dt*1e3:.1f} ms bad {bad} items {ctx.stat('prog_items')} "
                      f"chains {ctx.stat('prog_chains')}", {k: round(v, 2) for k, v in tm.items() if v > 0.05},
                      flush=True)


if __name__ == "__main__":
    main()
