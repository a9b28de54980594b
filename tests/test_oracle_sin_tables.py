"""The portable fdlibm `sin` (oracle `or_sin`, the same function the GPU's
k_coeffs evaluates) against glibc's `sin` (what fast_image_resize 5.5.0 calls
through Rust's f64::sin on Linux): the i16 Lanczos3 tables, bounds and
precisions of every pass crop_and_resize runs (image_processing.rs:288-323)
come out identical over the configs[1] and configs[2] size distributions.

resize_oracle.c states this equality; this test is its evidence.  A table
difference would be a real parity gap between the GPU and the reference, so
the test compares whole tables, not ULP distances."""
import ctypes

import numpy as np
import pytest

from oracle import buckets as B
from oracle import oracle as O

_libc = ctypes.CDLL(None)
_libc.free.argtypes = [ctypes.c_void_p]


class _Bound(ctypes.Structure):
    _fields_ = [("start", ctypes.c_int), ("size", ctypes.c_int)]


def _table(in_size, in0, in1, out_size, libm):
    L = O.lib()
    L.or_use_libm_sin.argtypes = [ctypes.c_int]
    L.or_coeffs.argtypes = [ctypes.c_int, ctypes.c_double, ctypes.c_double, ctypes.c_int, ctypes.c_int,
                            ctypes.POINTER(_Bound), ctypes.POINTER(ctypes.POINTER(ctypes.c_int32)),
                            ctypes.POINTER(ctypes.c_int)]
    L.or_coeffs.restype = ctypes.c_int
    L.or_use_libm_sin(1 if libm else 0)
    try:
        bounds = (_Bound * out_size)()
        cp = ctypes.POINTER(ctypes.c_int32)()
        prec = ctypes.c_int()
        k = L.or_coeffs(in_size, in0, in1, out_size, O.MODE_FIR, bounds, ctypes.byref(cp), ctypes.byref(prec))
        co = np.ctypeslib.as_array(cp, shape=(out_size * k,)).copy()
        _libc.free(ctypes.cast(cp, ctypes.c_void_p))
        bd = np.array([(b.start, b.size) for b in bounds], np.int32)
        return k, prec.value, bd, co
    finally:
        L.or_use_libm_sin(0)


def _passes(w, h, tw, th):
    """The (in_size, in0, in1, out_size) of every convolution crop_and_resize runs."""
    if (w, h) == (tw, th):
        return []
    nw, nh = B.scaled_size(w, h, tw, th)
    l, t, cw, ch = B.fit_crop_box(nw, nh, tw, th)
    out = []
    if nw != w:
        out.append((w, 0.0, float(w), nw))
    if nh != h:
        out.append((h, 0.0, float(h), nh))
    if l != int(l) or cw != tw:  # call 2: a fractional crop is a sub-pixel resample
        out.append((nw, l, l + cw, tw))
    if t != int(t) or ch != th:
        out.append((nh, t, t + ch, th))
    return out


def _sizes(config, n, seed):
    rng = np.random.default_rng(seed)
    if config == 1:  # configs[1]: AR log-uniform [0.4, 2.5], short side U[256, 2048]
        ar = np.exp(rng.uniform(np.log(0.4), np.log(2.5), n))
        short = rng.integers(256, 2049, n)
        return [(int(s * a), int(s)) if a >= 1 else (int(s), int(s / a)) for s, a in zip(short, ar)]
    return [(int(rng.integers(300, 501)), int(rng.integers(250, 501))) for _ in range(n)]  # configs[2]


@pytest.mark.parametrize("config,buckets,n", [(1, (1024, 32), 1500), (2, (512, 16), 1500)])
def test_fdlibm_and_glibc_sin_give_identical_tables(config, buckets, n):
    tr = B.ARAwareTransform(buckets[0], buckets[1], 0.5, 2.0)
    seen, checked = set(), 0
    for w, h in _sizes(config, n, 900 + config):
        for p in _passes(w, h, *tr.target_size(w, h)):
            if p in seen:
                continue
            seen.add(p)
            a, b = _table(*p, libm=False), _table(*p, libm=True)
            assert a[0] == b[0] and a[1] == b[1], p
            assert np.array_equal(a[2], b[2]) and np.array_equal(a[3], b[3]), p
            checked += 1
    assert checked > n  # call-1 H/V passes plus the x.5 crops
