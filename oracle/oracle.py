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
# JPEG decode semantics (jpeg_oracle.c oj_set_semantics): libjpeg-turbo (pinned
# against PIL) or zune-jpeg 0.5.12 restated (the reference's decoder; unpinned)
SEM_LIBJPEG, SEM_ZUNE = 0, 1

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
        L.oj_set_semantics.argtypes = [ctypes.c_int]
        L.oj_symbol_count.restype = ctypes.c_ulonglong
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


def set_semantics(mode: int) -> None:
    """JPEG decode semantics of every later jpeg_decode call (process-wide)."""
    lib().oj_set_semantics(mode)


class semantics:
    """with semantics(SEM_ZUNE): ... -- restores libjpeg-turbo mode on exit."""

    def __init__(self, mode: int):
        self.mode = mode

    def __enter__(self):
        set_semantics(self.mode)
        return self

    def __exit__(self, *exc):
        set_semantics(SEM_LIBJPEG)
        return False


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


# ------------------------------------------------------------------ PNG
PO_OK, PO_UNSUPPORTED, PO_CORRUPT, PO_SMALLBUF = 0, 1, 2, 3


def _png_lib():
    L = lib()
    if not getattr(L, "_png_ready", False):
        u8p = ctypes.POINTER(ctypes.c_uint8)
        ip = ctypes.POINTER(ctypes.c_int)
        L.po_info.argtypes = [u8p, ctypes.c_size_t] + [ip] * 6
        L.po_decode.argtypes = [u8p, ctypes.c_size_t, u8p, ctypes.c_size_t]
        L.po_zlib_inflate.argtypes = [u8p, ctypes.c_size_t, u8p, ctypes.c_size_t,
                                      ctypes.POINTER(ctypes.c_size_t)]
        L.po_premultiply.argtypes = [u8p, ctypes.c_size_t, ctypes.c_int]
        L.po_unpremultiply.argtypes = [u8p, ctypes.c_size_t, ctypes.c_int]
        L.po_blend_over_gray.argtypes = [u8p, ctypes.c_size_t, u8p]
        L._png_ready = True
    return L


def png_info(data: bytes):
    """(status, w, h, channels_after_expand, depth, color_type, interlace)."""
    v = [ctypes.c_int() for _ in range(6)]
    st = _png_lib().po_info(_u8(data), len(data), *[ctypes.byref(x) for x in v])
    return (st,) + tuple(x.value for x in v)


def png_decode(data: bytes):
    """Decode to HWC uint8 (C = 1..4 after EXPAND).  (status, array or None)."""
    st, w, h, c = png_info(data)[:4]
    if st != PO_OK:
        return st, None
    out = np.empty((h, w, c), np.uint8)
    st = _png_lib().po_decode(_u8(data), len(data), out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), out.nbytes)
    return st, (out if st == PO_OK else None)


def zlib_inflate(z: bytes, want: int):
    out = np.zeros(max(want, 1), np.uint8)
    got = ctypes.c_size_t()
    st = _png_lib().po_zlib_inflate(_u8(z), len(z), out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), want,
                                    ctypes.byref(got))
    return st, out[:got.value].tobytes()


def blend_over_gray(rgba: np.ndarray) -> np.ndarray:
    """convert_to_rgb8 for RGBA (image_processing.rs:163-186)."""
    rgba = np.ascontiguousarray(rgba, np.uint8)
    out = np.empty(rgba.shape[:-1] + (3,), np.uint8)
    _png_lib().po_blend_over_gray(rgba.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), rgba.size // 4,
                                  out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)))
    return out


def decode_any(data: bytes):
    """JPEG or PNG by magic bytes: (status, HWC array)."""
    if data[:8] == b"\x89PNG\r\n\x1a\n":
        return png_decode(data)
    return jpeg_decode(data)


def to_rgb8(arr: np.ndarray, resized: bool) -> np.ndarray:
    """image_to_payload's img_to_rgb8 step (image_processing.rs:362-372) on the
    transformed image.  LumaA8 quirk: a resized U8x2 image comes
    back from image_to_dyn_image as a GrayImage over the LA bytes, so its RGB
    is the first w*h bytes of the LA buffer as luma; an unresized LumaA8 drops
    its alpha."""
    h, w, c = arr.shape
    if c == 3:
        return arr
    if c == 4:
        return blend_over_gray(arr)
    if c == 2 and resized:
        g = np.ascontiguousarray(arr).reshape(-1)[: w * h].reshape(h, w)
    else:
        g = arr[:, :, 0]
    return np.repeat(g[:, :, None], 3, axis=2)


# ------------------------------------------------------------------ JPEG encode
def _enc_lib():
    L = lib()
    if not getattr(L, "_enc_ready", False):
        u8p = ctypes.POINTER(ctypes.c_uint8)
        L.oe_encode.argtypes = [u8p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, u8p, ctypes.c_size_t]
        L.oe_encode.restype = ctypes.c_size_t
        L.oe_bound.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int]
        L.oe_bound.restype = ctypes.c_size_t
        L.oe_qtables.argtypes = [ctypes.c_int, u8p]
        L.oe_fdct.argtypes = [u8p, ctypes.POINTER(ctypes.c_int32)]
        L._enc_ready = True
    return L


def jpeg_encode(arr: np.ndarray, quality: int = 92) -> bytes:
    """image 0.25 JpegEncoder::new_with_quality restated (image_processing.rs:374-395)."""
    arr = np.ascontiguousarray(arr, np.uint8)
    if arr.ndim == 2:
        arr = arr[:, :, None]
    h, w, c = arr.shape
    L = _enc_lib()
    cap = L.oe_bound(w, h, c)
    out = np.empty(cap, np.uint8)
    n = L.oe_encode(arr.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), w, h, c, quality,
                    out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), cap)
    assert n > 0
    return out[:n].tobytes()


def jpeg_qtables(quality: int) -> np.ndarray:
    q = np.empty((2, 64), np.uint8)
    _enc_lib().oe_qtables(quality, q.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)))
    return q


def jpeg_encode_bound(w: int, h: int, c: int) -> int:
    return int(_enc_lib().oe_bound(w, h, c))
