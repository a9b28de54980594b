"""Process-exit safety (tests/test_gpu_exit.py): leave the library busy and
exit without closing anything, the way a loader process ends when its
workers still own contexts (the Rust drop-in's
`Drop for GpuImageStage` may never run at exit).

What is left behind at exit:
  * two contexts, one with persistent planning workers (`plan_threads`);
  * `dg_decode_one` coalescing from several threads (joined, batches done);
  * a progressive aggregate still open: a submission whose progressive
    member was only `dg_wait_ready`-ed (never `dg_wait`-ed);
  * a device-resident batch submitted and never waited for;
  * reference cycles holding the contexts, so `__del__` does not run them
    down in order.

    exit_worker.py MODE   MODE: "atexit" (the Python close-all runs) or
                                "raw" (DG_NO_ATEXIT_CLOSE: nothing closes
                                the contexts; the library's own exit hook
                                must make the runtime's teardown safe)
Prints "EXIT-WORKER-OK" before returning from main; the parent checks rc 0."""
import os
import sys
import threading

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(mode: str) -> int:
    if mode == "raw":
        os.environ["DG_NO_ATEXIT_CLOSE"] = "1"
    import numpy as np

    from datago_amd import _lib as L
    from datago_amd import synth
    kw = dict(crop_and_resize=True, default_image_size=512, downsampling_ratio=16, min_aspect_ratio=0.5,
              max_aspect_ratio=2.0, decode_semantics=1)
    a = L.Context(0, **kw)
    a.set_option("plan_threads", 4)
    b = L.Context(0, **kw)
    datas = [synth.make_jpeg(100 + i, 320 + 16 * i, 240 + 8 * i, 85, "4:2:0") for i in range(24)]
    prog = synth.make_jpeg(999, 900, 700, 90, "4:2:0", progressive=True)
    # decode_one from threads (coalesced batches)
    errs = []

    def worker(k):
        for d in datas[k::6]:
            st, arr, m = a.decode_one(d)
            if st != 0:
                errs.append(st)
    ts = [threading.Thread(target=worker, args=(k,)) for k in range(6)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errs, errs
    # a big submission through the planning workers, completed
    res = a.decode_batch(datas * 4)
    assert all(st == 0 for st, _, _ in res)
    # a split submission: the baseline part finishes, the progressive member
    # stays in the open aggregate (no dg_wait)
    outs = [np.empty(max(b.output_size(d)[1], 1), np.uint8) for d in datas[:4] + [prog]]
    ticket, metas, keep = b.submit_host(datas[:4] + [prog], outs)
    pend = b.wait_ready(ticket)
    # a device-resident batch left in flight
    coded = b"".join(datas[:8])
    d_in = b.alloc(len(coded) + 64)
    b.h2d(d_in, np.frombuffer(coded, np.uint8))
    offs = np.cumsum([0] + [len(d) for d in datas[:7]])
    sizes = [b.output_size(d)[1] for d in datas[:8]]
    d_out = [b.alloc(s) for s in sizes]
    host = [np.frombuffer(d, np.uint8).ctypes.data for d in datas[:8]]
    t2, metas2 = b.submit_device(host, [d_in + int(o) for o in offs], [len(d) for d in datas[:8]], d_out, sizes)
    # reference cycles: the contexts outlive module teardown's refcount drops
    cyc_a, cyc_b = [a], [b]
    cyc_a.append(cyc_a)
    cyc_b.append(cyc_b)
    globals()["_keep"] = (cyc_a, cyc_b, outs, metas, keep, metas2)
    print("EXIT-WORKER-OK pending=%d" % pend, flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1] if len(sys.argv) > 1 else "atexit"))
