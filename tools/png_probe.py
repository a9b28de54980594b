"""PNG stage probe: the bench's configs[4] pairs split into masks only and
images only, each decoded in isolation (one batch in flight) and together,
so a kernel trace (rocprofv3 --kernel-trace) separates the serial mask
inflate from the chunked image path.  Wall times include the host copies
(decode_batch is the host-in/host-out path): read the kernel trace.

    python tools/png_probe.py [n_pairs] [reps] [opt=value ...] [--variants 2,8,9]

--variants: the images batch again under each inf_decode value (the variants
are distinct kernel instantiations, so one trace separates them).
"""
import sys
import time

sys.path.insert(0, ".")

import bench  # noqa: E402
from datago_amd import _lib as L  # noqa: E402

args = [a for a in sys.argv[1:] if not a.startswith("--variants")]
variants = [a.split("=", 1)[1] for a in sys.argv[1:] if a.startswith("--variants=")]
variants = [int(v) for v in variants[0].split(",")] if variants else []
n = int(args[0]) if len(args) > 0 else 128
reps = int(args[1]) if len(args) > 1 else 3
opts = [a.split("=") for a in args[2:]]
pool = bench.png_corpus(5, n, 256, 2048, 16, 0, n)
imgs, masks = pool[0::2], pool[1::2]


def ctx(extra=()):
    c = L.Context(0, crop_and_resize=True, default_image_size=1024, downsampling_ratio=32, min_aspect_ratio=0.5,
                  max_aspect_ratio=2.0, decode_semantics=1)
    for k, v in list(opts) + list(extra):
        c.set_option(k, int(v))
    return c


def run(c, name, batch):
    c.decode_batch(batch)
    ts = []
    for _ in range(reps):
        t = time.perf_counter()
        out = c.decode_batch(batch)
        ts.append((time.perf_counter() - t) * 1e3)
        assert all(s == 0 for s, _, _ in out)
    print(f"{name:7s} n={len(batch)} ms={min(ts):.1f} ({', '.join(f'{x:.1f}' for x in ts)}) "
          f"chunks={c.stat('png_chunks')} serial_fallbacks={c.stat('png_serial_fallbacks')} "
          f"small={c.stat('png_small_streams')}", flush=True)


c = ctx()
for name, batch in (("masks", masks), ("images", imgs), ("pairs", pool)):
    run(c, name, batch)
c.close()
for v in variants:
    c = ctx([("inf_decode", v)])
    run(c, f"img_v{v}", imgs)
    c.close()
