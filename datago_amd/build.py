"""Build libdatago_hip.so in-tree with hipcc for gfx950 (no torch extension
machinery: the library is a plain C-ABI shared object).

    python -m datago_amd.build [--jobs N] [--force]
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
BUILD = os.path.join(HERE, "_build")
LIB = os.path.join(HERE, "libdatago_hip.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("DG_OFFLOAD_ARCH", "gfx950")

SOURCES = [
    # (source, is_device_code)
    ("kernels.hip", True),
    ("dg_png.hip", True),
    ("dg_enc.hip", True),
    ("dg_prog.hip", True),
    ("dg_penc.hip", True),
    ("dg_band.hip", True),
    ("host/jpeg_enc.cpp", False),
    ("host/wds.cpp", False),
    ("host/png_header.cpp", False),
    ("host/pipeline.cpp", False),
    ("host/capi.cpp", False),
    ("host/jpeg_header.cpp", False),
    ("host/buckets.cpp", False),
]

COMMON = ["-O3", "-fPIC", "-std=c++17", "-ffp-contract=off", "-Wall", "-Wno-unused-function",
          f"-I{CSRC}", f"-I{os.path.join(ROOT, 'include')}"] + os.environ.get("DG_HIPCC_FLAGS", "").split()


def _obj(src: str) -> str:
    return os.path.join(BUILD, src.replace("/", "_") + ".o")


def _deps_newer(src: str, obj: str) -> bool:
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    paths = [os.path.join(CSRC, src)]
    for d in (CSRC, os.path.join(CSRC, "host"), os.path.join(ROOT, "include")):
        paths += [os.path.join(d, f) for f in os.listdir(d) if f.endswith(".h")]
    return any(os.path.getmtime(p) > t for p in paths)


def _compile(src: str, device: bool, force: bool) -> str:
    obj = _obj(src)
    if not force and not _deps_newer(src, obj):
        return obj
    if device:
        cmd = [HIPCC] + COMMON + [f"--offload-arch={ARCH}", "-x", "hip"]
    else:
        cmd = [HIPCC] + COMMON + ["-I/opt/rocm/include", "-x", "c++", "-D__HIP_PLATFORM_AMD__"]
    cmd += ["-c", os.path.join(CSRC, src), "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return obj


def build(force: bool = False, jobs: int = 4) -> str:
    os.makedirs(BUILD, exist_ok=True)
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        objs = list(ex.map(lambda s: _compile(s[0], s[1], force), SOURCES))
    newest = max(os.path.getmtime(o) for o in objs)
    if force or not os.path.exists(LIB) or os.path.getmtime(LIB) < newest:
        cmd = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", LIB] + objs + \
              ["-Wl,--no-undefined", "-Wl,-soname,libdatago_hip.so"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return LIB


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--jobs", type=int, default=4)
    a = ap.parse_args()
    print(build(a.force, a.jobs))
    return 0


if __name__ == "__main__":
    sys.exit(main())
