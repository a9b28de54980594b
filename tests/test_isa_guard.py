"""Compiler guard (DESIGN.md §3, gfx950 notes): hipcc 7.2 for gfx950 can fuse
a clamp-and-shift-and-pack of bytes into v_ashr_pk_u8_i32 and then OR the next
byte into that instruction's stale upper half, corrupting every third output
byte.  The kernels pack bytes with v_perm (pack4) instead; this test compiles
every device source for gfx950 and fails if the instruction reappears."""
import concurrent.futures as cf
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "datago_amd", "csrc")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
SOURCES = ["kernels.hip", "dg_png.hip", "dg_enc.hip", "dg_prog.hip", "dg_penc.hip"]


def _asm(src, tmp):
    out = os.path.join(tmp, src + ".s")
    subprocess.run([HIPCC, "-O3", "-std=c++17", "-ffp-contract=off", f"-I{CSRC}", f"-I{os.path.join(ROOT, 'include')}",
                    "--offload-arch=gfx950", "-x", "hip", "--cuda-device-only", "-S", os.path.join(CSRC, src),
                    "-o", out], check=True, capture_output=True)
    with open(out) as f:
        return src, f.read()


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not installed")
def test_no_v_ashr_pk_u8_i32(tmp_path):
    with cf.ThreadPoolExecutor(len(SOURCES)) as ex:
        for src, asm in ex.map(lambda s: _asm(s, str(tmp_path)), SOURCES):
            bad = [l for l in asm.splitlines() if "v_ashr_pk_u8_i32" in l or "v_lshr_pk_u8" in l]
            assert not bad, (src, bad[:3])

