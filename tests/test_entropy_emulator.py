"""The GPU entropy decoder's algorithm (datago_amd/csrc/dg_entropy.h — the
product's own decode_range()) emulated sequentially on the CPU with the phase
structure of k_huff_sync / k_huff_fix / k_huff_scan / k_huff_write, checked
bit-exactly against the oracle's coefficients.  Catches logic errors in the
self-synchronising decode without a GPU."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

from datago_amd import synth
from oracle import oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NATIVE = os.path.join(ROOT, "tests", "native")
SO = os.path.join(NATIVE, "libemu.so")


@pytest.fixture(scope="module")
def emu():
    srcs = [os.path.join(NATIVE, "emu.cpp"), os.path.join(ROOT, "datago_amd", "csrc", "host", "jpeg_header.cpp")]
    deps = srcs + [os.path.join(ROOT, "datago_amd", "csrc", f) for f in ("dg_entropy.h", "dg_types.h")]
    if not os.path.exists(SO) or any(os.path.getmtime(p) > os.path.getmtime(SO) for p in deps):
        # build beside it and rename: parallel test workers never load a half-written library
        tmp = f"{SO}.{os.getpid()}.tmp"
        subprocess.run(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off",
                        "-I" + os.path.join(ROOT, "datago_amd", "csrc"), "-o", tmp] + srcs, check=True)
        os.replace(tmp, SO)
    E = ctypes.CDLL(SO)
    E.emu_set_lead.argtypes = [ctypes.c_uint32]
    E.emu_decode_coefs.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_uint32,
                                   ctypes.POINTER(ctypes.c_int16), ctypes.c_size_t,
                                   ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(ctypes.c_int64)]

    E.emu_multi_mismatch.restype = ctypes.c_int64
    E.emu_multi_checked.restype = ctypes.c_int64
    E.emu_two_mismatch.restype = ctypes.c_int64
    E.emu_two_checked.restype = ctypes.c_int64

    def run(data, sub_bits, lead=0):
        E.emu_set_lead(lead)
        run.multi0 = (E.emu_multi_mismatch(), E.emu_multi_checked())
        run.two0 = (E.emu_two_mismatch(), E.emu_two_checked())
        cap = 1 << 18
        out = np.zeros((cap, 64), np.int16)
        nb = ctypes.c_size_t()
        st = (ctypes.c_int64 * 8)()
        r = E.emu_decode_coefs(data, len(data), sub_bits, out.ctypes.data_as(ctypes.POINTER(ctypes.c_int16)),
                               cap, ctypes.byref(nb), st)
        run.multi = (E.emu_multi_mismatch() - run.multi0[0], E.emu_multi_checked() - run.multi0[1])
        run.two = (E.emu_two_mismatch() - run.two0[0], E.emu_two_checked() - run.two0[1])
        return r, out[: nb.value], list(st)
    return run


@pytest.mark.parametrize("seed", range(24))
@pytest.mark.parametrize("sub_bits,lead", [(128, 0), (1024, 0), (4096, 0), (512, 96), (1024, 2048), (4096, 6144)])
def test_emulated_parallel_decode_matches_oracle(emu, seed, sub_bits, lead):
    rng = np.random.default_rng(seed)
    w, h = int(rng.integers(1, 700)), int(rng.integers(1, 700))
    ss = ["4:2:0", "4:2:2", "4:4:4"][seed % 3]
    rst = [0, 0, 1, 3][seed % 4]
    data = synth.encode_jpeg(synth.synth_pixels(rng, w, h, seed % 7 == 0), int(rng.integers(30, 101)), ss,
                             restart_marker_rows=rst)
    st, ref = O.jpeg_coefs(data)
    r, co, stats = emu(data, sub_bits, lead)
    assert r == 0 and st == 0
    assert co.shape == ref.shape
    assert np.array_equal(co, ref)
    assert stats[5] == 0  # write pass exit == next subsequence's entry everywhere
    # k_huff_sync's multi-symbol lead-in (kMultiBits lookups) ends in the same state as single steps
    assert emu.multi[0] == 0, emu.multi
    # k_huff_sync2: two chains per lane in lockstep equal lead_in + decode_range per slot
    assert emu.two[0] == 0 and emu.two[1] > 0, emu.two


def test_truncated_stream_is_detected(emu):
    data = synth.make_jpeg(3, 300, 200, 90, "4:2:0")
    cut = data[: len(data) * 2 // 3]
    r, co, stats = emu(cut, 1024)
    assert stats[6] < stats[7]  # decoded blocks < total blocks -> CORRUPT on the GPU path
