"""ORACLE — test infrastructure only.

ctypes loader for oracle/liboracle.so (the C restatements in this directory).
Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import it.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from typing import Tuple

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")

OJ_OK, OJ_UNSUPPORTED, OJ_CORRUPT, OJ_SMALLBUF = 0, 1, 2, 3
MODE_FIR, MODE_PILLOW = 0, 1

_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        u8p = ctypes.POINTER(ctypes.c_uint8)
        ip = ctypes.POINTER(ctypes.c_int)
        L.oj_info.argtypes = [u8p, ctypes.c_size_t, ip, ip, ip]
        L.oj_decode.argtypes = [u8p, ctypes.c_size_t, u8p, ctypes.c_size_t, ip, ip, ip]
        L.oj_decode_coefs.argtypes = [u8p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_int16),
                                      ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t)]
        L.or_crop_and_resize.argtypes = [u8p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                         ctypes.c_int, ctypes.c_int, u8p, ctypes.c_int]
        L.or_resample.argtypes = [u8p, ctypes.c_int, ctypes.c_int, ctypes.c_int, u8p,
                                  ctypes.c_int, ctypes.c_int, ctypes.c_double, ctypes.c_double,
                                  ctypes.c_double, ctypes.c_double, ctypes.c_int]
        L.or_scaled_size.argtypes = [ctypes.c_int] * 4 + [ip, ip]
        dp = ctypes.POINTER(ctypes.c_double)
        L.or_fit_crop.argtypes = [ctypes.c_int] * 4 + [dp] * 4
        _lib = L
    return _lib


def _u8(buf) -> ctypes.POINTER(ctypes.c_uint8):
    return ctypes.cast(ctypes.c_char_p(bytes(buf)), ctypes.POINTER(ctypes.c_uint8))


def jpeg_info(data: bytes) -> Tuple[int, int, int, int]:
    w, h, nc = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    st = lib().oj_info(_u8(data), len(data), ctypes.byref(w), ctypes.byref(h), ctypes.byref(nc))
    return st, w.value, h.value, nc.value


def jpeg_decode(data: bytes) -> Tuple[int, np.ndarray]:
    """Decode to HWC uint8 (C=1 or 3).  Returns (status, array or None)."""
    st, w, h, nc = jpeg_info(data)
    if st != OJ_OK:
        return st, None
    out = np.empty((h, w, nc), np.uint8)
    ww, hh, cc = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    st = lib().oj_decode(_u8(data), len(data), out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)),
                         out.nbytes, ctypes.byref(ww), ctypes.byref(hh), ctypes.byref(cc))
    return st, (out if st == OJ_OK else None)


def jpeg_coefs(data: bytes, max_blocks: int = 1 << 20) -> Tuple[int, np.ndarray]:
    """Quantized coefficients in decode order, shape (nblocks, 64), natural order."""
    out = np.zeros((max_blocks, 64), np.int16)
    nb = ctypes.c_size_t()
    st = lib().oj_decode_coefs(_u8(data), len(data),
                               out.ctypes.data_as(ctypes.POINTER(ctypes.c_int16)), max_blocks,
                               ctypes.byref(nb))
    return st, out[: nb.value].copy()


def resample(src: np.ndarray, dw: int, dh: int, box, mode: int = MODE_FIR) -> np.ndarray:
    src = np.ascontiguousarray(src)
    if src.ndim == 2:
        src = src[:, :, None]
    h, w, c = src.shape
    out = np.empty((dh, dw, c), np.uint8)
    x0, y0, x1, y1 = box
    lib().or_resample(src.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), w, h, c,
                      out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), dw, dh,
                      float(x0), float(y0), float(x1), float(y1), mode)
    return out


def crop_and_resize(src: np.ndarray, tw: int, th: int, mode: int = MODE_FIR) -> np.ndarray:
    src = np.ascontiguousarray(src)
    if src.ndim == 2:
        src = src[:, :, None]
    h, w, c = src.shape
    out = np.empty((th, tw, c), np.uint8)
    lib().or_crop_and_resize(src.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), w, h, c, tw, th,
                             out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), mode)
    return out


def scaled_size(w: int, h: int, tw: int, th: int) -> Tuple[int, int]:
    a, b = ctypes.c_int(), ctypes.c_int()
    lib().or_scaled_size(w, h, tw, th, ctypes.byref(a), ctypes.byref(b))
    return a.value, b.value


def fit_crop(sw: int, sh: int, dw: int, dh: int):
    v = [ctypes.c_double() for _ in range(4)]
    lib().or_fit_crop(sw, sh, dw, dh, *[ctypes.byref(x) for x in v])
    return tuple(x.value for x in v)
