"""Device memory budget (context option max_device_mb).

A submission whose plan does not fit the budget is split into sub-batches
under the caller's one ticket; the outputs stay bit-exact (equal to an
unbudgeted context's, which the parity suites pin to the oracle).  An image
that alone exceeds the budget fails with DG_ERR_OOM and nothing else does
(worker_files.rs:63-70: a failed sample is dropped, never the worker)."""
import numpy as np
import pytest

from datago_amd import _lib as L
from datago_amd import synth

pytestmark = pytest.mark.gpu

KW = dict(crop_and_resize=True, default_image_size=512, downsampling_ratio=16, min_aspect_ratio=0.5,
          max_aspect_ratio=2.0, decode_semantics=1)


def _ctx():
    """A context without the Lanczos table cache (its arena would not count
    the same with and without a budget)."""
    c = L.Context(0, **KW)
    c.set_option("coef_cache_mb", 0)
    return c


def _base_mb():
    """Device MB of a context after one tiny image: table pools + tiny arenas
    (allocated as a budgeted context does: exact sizes, no growth headroom;
    budget_plan 0: a huge budget would otherwise be planned for)."""
    c = _ctx()
    c.set_option("budget_plan", 0)
    c.set_option("max_device_mb", 1 << 20)
    st, _, _ = c.decode_batch([synth.make_jpeg(1, 32, 32, 90)])[0]
    assert st == 0
    mb = c.stat("device_mb")
    c.close()
    return mb


def _ref_ctx():
    """Unbudgeted outputs, footprint as one slot's exact-size buffers (a huge
    budget: no growth headroom, no prewarmed idle slots)."""
    c = _ctx()
    c.set_option("budget_plan", 0)
    c.set_option("max_device_mb", 1 << 20)
    return c


def test_budget_splits_stay_bit_exact():
    datas = synth.mixed_corpus(77, 40, 256, 1200)
    ref = _ref_ctx()
    want = ref.decode_batch(datas)
    peak = ref.stat("peak_device_mb")
    ref.close()
    base = _base_mb()
    assert peak > base
    budget = base + max(8, (peak - base) // 3)
    c = _ctx()
    c.set_option("max_device_mb", budget)
    got = c.decode_batch(datas)
    assert c.stat("budget_splits") > 0, (peak, base, budget)
    for (s0, a0, _), (s1, a1, _) in zip(want, got):
        assert s0 == s1 == 0
        assert a0.shape == a1.shape and np.array_equal(a0, a1)
    # the descriptor buffer grows after the budget check: a few MB of slack at most
    assert c.stat("peak_device_mb") <= budget + 16, (c.stat("peak_device_mb"), budget)
    # device-resident submissions under the same budget: one ticket, several parts
    tk, metas, keep = c.submit_host(datas[:12], [np.empty(max(c.output_size(d)[1], 1), np.uint8)
                                                 for d in datas[:12]])
    c.wait(tk)
    assert all(metas[i].status == 0 for i in range(12))
    c.close()


def test_image_over_budget_fails_alone():
    base = _base_mb()
    c = _ctx()
    c.set_option("max_device_mb", base + 6)
    small = [synth.make_jpeg(10 + i, 96, 64, 90) for i in range(3)]
    big = synth.make_jpeg(20, 2400, 1800, 92)
    res = c.decode_batch(small[:2] + [big] + small[2:])
    assert [r[0] for r in res] == [0, 0, L.DG_ERR_OOM, 0]
    assert c.stat("budget_oom") == 1
    ok = _ctx()
    for (s, a, _), (s2, a2, _) in zip([res[0], res[1], res[3]], ok.decode_batch(small)):
        assert s == s2 == 0 and np.array_equal(a, a2)
    ok.close()
    c.close()


def test_budget_with_progressive_members():
    """A split submission with progressive members: the baseline part splits,
    the aggregate too; dg_wait_ready then dg_wait complete every member."""
    base = _base_mb()
    datas = synth.mixed_corpus(78, 16, 256, 900)
    datas[3] = synth.make_jpeg(31, 700, 500, 90, "4:2:0", progressive=True)
    datas[9] = synth.make_jpeg(32, 500, 700, 90, "4:4:4", progressive=True)
    ref = _ref_ctx()
    want = ref.decode_batch(datas)
    peak = ref.stat("peak_device_mb")
    ref.close()
    c = _ctx()
    c.set_option("max_device_mb", base + max(8, (peak - base) // 3))
    outs = [np.zeros(max(c.output_size(d)[1], 1), np.uint8) for d in datas]
    tk, metas, keep = c.submit_host(datas, outs)
    c.wait_ready(tk)
    c.wait(tk)
    for i, (s0, a0, _) in enumerate(want):
        assert s0 == 0 and metas[i].status == 0
        assert np.array_equal(outs[i][: a0.size], a0.reshape(-1))
    c.close()


def test_budget_settles_on_fewer_slots():
    """A budget that holds ~2.5 slots' buffers: the context takes slots out of
    turn (stat budget_slots) instead of trading buffers between slots batch
    after batch; 12 batches in flight stay bit-exact."""
    datas = synth.mixed_corpus(79, 12, 256, 900)
    ref = _ctx()
    want = ref.decode_batch(datas)
    ref.close()
    base = _base_mb()
    one = _ctx()
    one.set_option("budget_plan", 0)
    one.set_option("max_device_mb", 1 << 20)  # exact sizes, as under a budget
    one.decode_batch(datas)
    per_slot = one.stat("device_mb") - base
    one.close()
    assert per_slot > 0
    budget = base + (5 * per_slot) // 2
    c = _ctx()
    c.set_option("max_device_mb", budget)
    runs = []
    for _ in range(12):
        outs = [np.zeros(max(c.output_size(d)[1], 1), np.uint8) for d in datas]
        runs.append((c.submit_host(datas, outs), outs))
    for (tk, metas, keep), outs in runs:
        c.wait(tk)
        for i, (s0, a0, _) in enumerate(want):
            assert s0 == 0 and metas[i].status == 0
            assert np.array_equal(outs[i][: a0.size], a0.reshape(-1))
    assert c.stat("budget_slots") <= 3, c.stat("budget_slots")
    assert c.stat("budget_frees") <= 8, c.stat("budget_frees")  # a few slots given back once, not per batch
    assert c.stat("budget_oom") == 0
    assert c.stat("peak_device_mb") <= budget + 16, (c.stat("peak_device_mb"), budget)
    c.close()


def test_split_failure_waits_for_launched_parts():
    """a budget split whose second part fails after the first
    launched returns the error only once the launched part has finished
    writing the caller's outputs (host-out: copied back), so the caller may
    free its buffers as soon as the call fails; the context stays usable."""
    datas = synth.mixed_corpus(78, 24, 256, 1200)
    ref = _ref_ctx()
    ref.decode_batch(datas)
    peak = ref.stat("peak_device_mb")
    ref.close()
    base = _base_mb()
    c = _ctx()
    c.set_option("max_device_mb", base + max(8, (peak - base) // 3))
    c.set_option("debug_flags", 1 << 24)
    outs = [np.empty(max(c.output_size(d)[1], 1), np.uint8) for d in datas]
    with pytest.raises(L.DgError) as e:
        c.submit_host(datas, outs)
    assert "second part" in str(e.value)
    assert c.stat("budget_splits") > 0
    del outs  # the launched part is finished: freeing the outputs is safe
    c.set_option("debug_flags", 0)
    got = c.decode_batch(datas)
    assert all(s == 0 for s, _, _ in got)
    c.close()


def test_planned_budget_allocates_nothing_after_first_batch():
    """under a budget the first batch decides the slot count
    and sizes every slot it will use (option budget_plan, default on); later
    batches -- several in flight, cycling over the slots -- allocate and free
    nothing (stats allocs / budget_frees unchanged), stay within the budget
    and bit-exact against an unbudgeted context."""
    # the first batch holds the largest files: every later batch fits the
    # pinned staging and descriptor buffers it sized (their growth would be an
    # allocation too)
    datas = sorted(synth.mixed_corpus(79, 48, 256, 1100), key=len, reverse=True)
    batches = [datas[i:i + 8] for i in range(0, 48, 8)]
    ref = _ref_ctx()
    want = [ref.decode_batch(b) for b in batches]
    one = ref.stat("peak_device_mb")
    ref.close()
    base = _base_mb()
    budget = base + 3 * max(8, one - base)
    c = _ctx()
    c.set_option("max_device_mb", budget)
    outs = [[np.empty(max(c.output_size(d)[1], 1), np.uint8) for d in b] for b in batches]
    tk, metas, keep = c.submit_host(batches[0], outs[0])
    c.wait(tk)
    a0, f0 = c.stat("allocs"), c.stat("budget_frees")
    assert c.stat("budget_slots") >= 2, (c.stat("budget_slots"), budget, one, base)
    for rep in range(2):
        pend = []
        for k, b in enumerate(batches):
            pend.append((k, c.submit_host(b, outs[k])))
            if len(pend) >= 3:
                k0, (t0, m0, _) = pend.pop(0)
                c.wait(t0)
        for k0, (t0, m0, _) in pend:
            c.wait(t0)
        for k, b in enumerate(batches):
            for j, (st, arr, _) in enumerate(want[k]):
                assert st == 0 and np.array_equal(outs[k][j][:arr.size].reshape(arr.shape), arr), (rep, k, j)
    assert c.stat("allocs") == a0, (a0, c.stat("allocs"))
    assert c.stat("budget_frees") == f0
    assert c.stat("budget_splits") == 0
    assert c.stat("peak_device_mb") <= budget, (c.stat("peak_device_mb"), budget)
    c.close()
