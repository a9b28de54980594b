"""C-ABI library: loads, exports every symbol include/datago_hip.h declares,
and its host-only entry points (buckets, probe) agree with the oracle.  No
compute calls: these run without a GPU."""
import ctypes
import json
import os
import re
import subprocess

import pytest

from datago_amd import _lib
from datago_amd import synth
from oracle import buckets as B

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "include", "datago_hip.h")


@pytest.fixture(scope="module")
def L():
    if not os.path.exists(_lib.LIB_PATH):
        from datago_amd import build
        build.build()
    return _lib.load()


def _header_functions():
    src = open(HDR).read()
    return sorted(set(re.findall(r"\b(dg_[a-z0-9_]+)\(", src)))


def test_every_declared_symbol_is_exported(L):
    declared = _header_functions()
    assert len(declared) >= 25
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r" T (dg_\w+)", out))
    missing = [f for f in declared if f not in exported]
    assert not missing, missing
    assert sorted(_lib.EXPORTS) == declared


def test_no_torch_types_in_abi():
    src = open(HDR).read()
    assert "torch" not in src.lower() and "at::" not in src and "hip_runtime" not in src


def test_abi_version(L):
    assert L.dg_abi_version() == 3  # 2: dg_image_config.decode_semantics; 3: dg_wait_ready


@pytest.mark.parametrize("cfg", list(B.CONFIGS.keys()))
def test_bucket_table_matches_oracle(L, cfg):
    size, ratio, lo, hi = B.CONFIGS[cfg]
    t = _lib.BucketTable(size, ratio, lo, hi)
    o = B.ARAwareTransform(size, ratio, lo, hi)
    assert [k for _, k in o.aspect_ratios] == [b[2] for b in t.buckets()]
    assert [o.aspect_ratio_to_size[k] for _, k in o.aspect_ratios] == [(b[0], b[1]) for b in t.buckets()]
    with open(os.path.join(ROOT, "tests", "golden", "buckets.json")) as f:
        g = json.load(f)[cfg]
    for w, h, k in g["closest"]:
        assert t.get(t.closest(w, h))[2] == k
    for w in range(1, 3000, 37):
        for h in range(1, 3000, 53):
            assert t.get(t.closest(w, h))[2] == o.get_closest_aspect_ratio(w, h)


def test_reference_known_answers_through_abi(L):
    # image_processing.rs:441-478
    t = _lib.BucketTable(224, 16, 0.5, 2.0)
    assert t.get(t.closest(100, 100))[2] == "1.000"
    assert t.get(t.closest(200, 100))[2] == "1.900"
    assert t.get(t.closest(100, 200))[2] == "0.526"
    assert t.get(t.find_key("1.900"))[:2] == (304, 160)
    assert t.find_key("9.999") == -1  # the reference panics here (:334-336)
    assert _lib.aspect_ratio_to_str(150, 100) == "1.500"
    assert _lib.aspect_ratio_to_str(100, 200) == "0.500"


def test_invalid_config_is_a_status_not_an_abort(L):
    h = ctypes.c_void_p()
    assert L.dg_bucket_table_build(224, 0, 0.5, 2.0, ctypes.byref(h)) == _lib.DG_ERR_INVALID
    assert L.dg_bucket_table_build(224, 16, 2.0, 0.5, ctypes.byref(h)) == _lib.DG_ERR_INVALID


def test_probe(L):
    d = synth.make_jpeg(1, 123, 45, 90, "4:2:2")
    st, info = _lib.probe(d)
    assert st == 0 and info.format == _lib.DG_FMT_JPEG and (info.width, info.height) == (123, 45)
    assert info.components == 3 and info.gpu_supported == 1 and (info.h_samp[0], info.v_samp[0]) == (2, 1)
    st, info = _lib.probe(b"This is not a valid image file")
    assert st == _lib.DG_ERR_CORRUPT
    import io
    import numpy as np
    from PIL import Image
    buf = io.BytesIO()
    Image.fromarray(synth.synth_pixels(np.random.default_rng(0), 40, 30)).save(buf, format="JPEG", progressive=True)
    st, info = _lib.probe(buf.getvalue())
    assert st == 0 and info.progressive == 1 and info.gpu_supported == 1
    st, info = _lib.probe(synth.make_cmyk_jpeg(0, 40, 30))
    assert st == 0 and info.components == 4 and info.gpu_supported == 0
    buf = io.BytesIO()
    Image.new("RGB", (7, 5)).save(buf, format="PNG")
    st, info = _lib.probe(buf.getvalue())
    assert st == 0 and info.format == _lib.DG_FMT_PNG and (info.width, info.height) == (7, 5)


def test_probe_accepts_more_than_64_progressive_scans(L):
    """The header parser takes up to 256 scans (the deps-mask cap
    of 64 no longer refuses files; such files run chained on the GPU)."""
    import ctypes
    from test_gpu_progressive import _many_scan_jpeg
    d = _many_scan_jpeg(9100)
    assert d.count(b"\xff\xda") == 65
    info = _lib.ProbeInfo()
    assert L.dg_probe(d, len(d), ctypes.byref(info)) == 0
    assert info.progressive == 1 and info.gpu_supported == 1


def test_failing_calls_set_last_error(L):
    """dg_last_error names the failure of the call that just failed (VERDICT r5
    item 8), also for calls that need no GPU: a null context or key."""
    assert L.dg_ctx_set_option(None, b"slots", 4) == _lib.DG_ERR_INVALID
    assert _lib.last_error() == "null context"
    h = ctypes.c_void_p()
    assert L.dg_bucket_table_build(224, 0, 0.5, 2.0, ctypes.byref(h)) == _lib.DG_ERR_INVALID
    assert _lib.last_error() == "invalid bucket parameters"
    assert L.dg_ctx_get_stat(None, b"batches") == -1
    assert _lib.last_error() == "null context"
