import sys; sys.path.insert(0, '/root/repo'); sys.path.insert(0, '/root/repo/tests')
import numpy as np
from datago_amd import _lib as L, synth
import test_gpu_budget as T
datas = synth.mixed_corpus(77, 40, 256, 1200)
ref = T._ref_ctx(); ref.decode_batch(datas); peak = ref.stat("peak_device_mb"); ref.close()
base = T._base_mb()
budget = base + max(8, (peak - base) // 3)
print("base", base, "peak", peak, "budget", budget)
c = T._ctx(); c.set_option("max_device_mb", budget)
got = c.decode_batch(datas)
for k in ("peak_device_mb", "device_mb", "budget_slots", "budget_splits", "budget_plan_mb", "allocs", "budget_frees", "hpool", "qpool"):
    print(k, c.stat(k))
