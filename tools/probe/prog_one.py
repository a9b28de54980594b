"""Decode the configs[1] pool's largest progressive file (PMC target): one
launch per level (prog_pipe 0), so the final luma refinement scan is a
dispatch of its own."""
import os
import sys

sys.path.insert(0, ".")
from datago_amd import synth  # noqa: E402
from datago_amd import _lib as L  # noqa: E402

spec = synth.mixed_spec(2, 256, 256, 2048)
i = max(range(256), key=lambda j: spec[j][0] * spec[j][1])
w, h, q, ss, g = spec[i]
data = synth.make_jpeg(2 * 1_000_003 + i, w, h, q, ss, g, 0, progressive=True)
ctx = L.Context(0)
ctx.set_option("progressive", 1)
ctx.set_option("prog_pipe", int(os.environ.get("PIPE", "0")))
for _ in range(int(os.environ.get("REPS", "2"))):
    st = ctx.decode_batch([data])[0][0]
    assert st == 0, st
print("ok", w, h, len(data), flush=True)
