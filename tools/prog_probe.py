"""Time the progressive scan kernel on single images (debug helper)."""
import sys
import time

import numpy as np

sys.path.insert(0, ".")
from datago_amd import synth  # noqa: E402
from datago_amd import _lib as L  # noqa: E402


def main():
    spec = synth.mixed_spec(2, 256, 256, 2048)
    big = sorted(range(256), key=lambda i: -spec[i][0] * spec[i][1])[:1]
    cases = []
    for i in big:
        w, h, q, ss, g = spec[i]
        cases.append(("pool-largest", synth.make_jpeg(2 * 1_000_003 + i, w, h, q, ss, g, 0, progressive=True)))
    cases.append(("1024x1024 q90", synth.make_jpeg(5, 1024, 1024, 90, progressive=True)))
    cases.append(("1024x1024 q90 baseline", synth.make_jpeg(5, 1024, 1024, 90)))
    for serial, pipe in ((1, 0), (0, 0), (0, 1)):
        ctx = L.Context(0)
        ctx.set_option("timing", 1)
        ctx.set_option("progressive", 1)
        ctx.set_option("prog_serial", serial)
        ctx.set_option("prog_pipe", pipe)
        run(ctx, cases, ("serial" if serial else "speculative") + ("+pipelined" if pipe else "+levels"))


def run(ctx, cases, mode):
    for name, d in cases:
        for rep in range(3):
            t = time.perf_counter()
            res = ctx.decode_batch([d])
            dt = time.perf_counter() - t
        tm = ctx.timings()
        print(mode, name, len(d), "status", res[0][0], f"wall {dt*1e3:.1f} ms",
              {k: round(v, 3) for k, v in tm.items() if v > 0.01}, flush=True)


if __name__ == "__main__":
    main()
