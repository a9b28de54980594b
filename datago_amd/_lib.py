"""ctypes binding of libdatago_hip.so (the C ABI in include/datago_hip.h).

The product path: every call goes to the HIP library.  There is no CPU
fallback — if the library is missing, importing this module raises.

torch (when installed) is imported first so that the process holds exactly one
HIP runtime: torch ships its own libamdhip64.so (soname libamdhip64.so.7) and
loads it via DT_NEEDED "libamdhip64.so"; our library's DT_NEEDED
"libamdhip64.so.7" then binds to that same copy instead of a second one.
"""
from __future__ import annotations

import atexit
import ctypes
import os
import weakref
from typing import List, Optional, Sequence, Tuple

import numpy as np

try:  # one HIP runtime per process (see module docstring)
    import torch  # noqa: F401
except Exception:  # pragma: no cover - torch is part of the image
    torch = None

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("DG_LIB_PATH") or os.path.join(HERE, "libdatago_hip.so")  # override: experiment builds

DG_OK, DG_ERR_UNSUPPORTED, DG_ERR_CORRUPT, DG_ERR_OOM, DG_ERR_BAD_BUCKET = 0, 1, 2, 3, 4
DG_ERR_INVALID, DG_ERR_SMALL_BUFFER, DG_ERR_DEVICE, DG_ERR_NOT_READY = 5, 6, 7, 8
STATUS_NAMES = {0: "OK", 1: "UNSUPPORTED", 2: "CORRUPT", 3: "OOM", 4: "BAD_BUCKET", 5: "INVALID",
                6: "SMALL_BUFFER", 7: "DEVICE", 8: "NOT_READY"}
DG_FMT_UNKNOWN, DG_FMT_JPEG, DG_FMT_PNG = 0, 1, 2

# exported symbols (must match include/datago_hip.h; checked by tests)
EXPORTS = [
    "dg_bucket_table_build", "dg_bucket_table_free", "dg_bucket_count", "dg_bucket_get",
    "dg_closest_bucket", "dg_bucket_find_key", "dg_aspect_ratio_to_str", "dg_probe",
    "dg_ctx_create", "dg_ctx_destroy", "dg_ctx_buckets", "dg_output_size", "dg_submit", "dg_wait",
    "dg_poll", "dg_wait_ready", "dg_decode_one", "dg_submit_device", "dg_device_alloc", "dg_device_free",
    "dg_memcpy_h2d", "dg_memcpy_d2h", "dg_synchronize", "dg_last_batch_timings",
    "dg_ctx_set_option", "dg_ctx_get_stat", "dg_last_error", "dg_abi_version", "dg_sample_align",
    "dg_wds_index", "dg_wds_key_hash", "dg_host_register", "dg_host_unregister",
]


class DgError(RuntimeError):
    def __init__(self, status: int, msg: str = ""):
        super().__init__(f"{STATUS_NAMES.get(status, status)}: {msg}")
        self.status = status


class ImageConfig(ctypes.Structure):
    _fields_ = [("crop_and_resize", ctypes.c_int32), ("default_image_size", ctypes.c_uint32),
                ("downsampling_ratio", ctypes.c_uint32), ("min_aspect_ratio", ctypes.c_double),
                ("max_aspect_ratio", ctypes.c_double), ("pre_encode_images", ctypes.c_int32),
                ("image_to_rgb8", ctypes.c_int32), ("encode_format", ctypes.c_int32),
                ("jpeg_quality", ctypes.c_int32), ("decode_semantics", ctypes.c_int32)]


class ProbeInfo(ctypes.Structure):
    _fields_ = [("format", ctypes.c_int32), ("width", ctypes.c_uint32), ("height", ctypes.c_uint32),
                ("components", ctypes.c_int32), ("bit_depth", ctypes.c_int32),
                ("h_samp", ctypes.c_int32 * 4), ("v_samp", ctypes.c_int32 * 4),
                ("progressive", ctypes.c_int32), ("arithmetic", ctypes.c_int32),
                ("precision", ctypes.c_int32), ("restart_interval", ctypes.c_int32),
                ("gpu_supported", ctypes.c_int32)]


class PayloadMeta(ctypes.Structure):
    _fields_ = [("original_width", ctypes.c_uint32), ("original_height", ctypes.c_uint32),
                ("width", ctypes.c_uint32), ("height", ctypes.c_uint32), ("channels", ctypes.c_int32),
                ("bit_depth", ctypes.c_int32), ("is_encoded", ctypes.c_int32), ("status", ctypes.c_int32),
                ("bucket", ctypes.c_int32), ("nbytes", ctypes.c_uint64)]


_lib: Optional[ctypes.CDLL] = None


def load() -> ctypes.CDLL:
    """Load the HIP library; raises if it has not been built (no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} not built: run `python -m datago_amd.build` "
                          "(the GPU path has no CPU fallback)")
    L = ctypes.CDLL(LIB_PATH)
    vp, sz, u8pp = ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_void_p)
    i32, u32, u64, dbl = ctypes.c_int32, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_double
    L.dg_bucket_table_build.argtypes = [u32, u32, dbl, dbl, ctypes.POINTER(vp)]
    L.dg_bucket_table_free.argtypes = [vp]
    L.dg_bucket_table_free.restype = None
    L.dg_bucket_count.argtypes = [vp]
    L.dg_bucket_get.argtypes = [vp, i32, ctypes.POINTER(u32), ctypes.POINTER(u32), ctypes.c_char_p, sz]
    L.dg_closest_bucket.argtypes = [vp, i32, i32]
    L.dg_bucket_find_key.argtypes = [vp, ctypes.c_char_p]
    L.dg_aspect_ratio_to_str.argtypes = [u32, u32, ctypes.c_char_p, sz]
    L.dg_probe.argtypes = [ctypes.c_char_p, sz, ctypes.POINTER(ProbeInfo)]
    L.dg_ctx_create.argtypes = [i32, ctypes.POINTER(ImageConfig), ctypes.POINTER(vp)]
    L.dg_ctx_destroy.argtypes = [vp]
    L.dg_ctx_destroy.restype = None
    L.dg_ctx_buckets.argtypes = [vp]
    L.dg_ctx_buckets.restype = vp
    L.dg_output_size.argtypes = [vp, ctypes.c_char_p, sz, i32, ctypes.POINTER(u64)]
    L.dg_submit.argtypes = [vp, i32, u8pp, ctypes.POINTER(sz), ctypes.POINTER(i32), u8pp,
                            ctypes.POINTER(u64), ctypes.POINTER(PayloadMeta), ctypes.POINTER(u64)]
    L.dg_submit_device.argtypes = [vp, i32, u8pp, u8pp, ctypes.POINTER(sz), ctypes.POINTER(i32), u8pp,
                                   ctypes.POINTER(u64), ctypes.POINTER(PayloadMeta), ctypes.POINTER(u64)]
    L.dg_wait.argtypes = [vp, u64]
    L.dg_poll.argtypes = [vp, u64]
    L.dg_wait_ready.argtypes = [vp, u64, ctypes.POINTER(i32)]
    L.dg_decode_one.argtypes = [vp, ctypes.c_char_p, sz, i32, vp, u64, ctypes.POINTER(PayloadMeta)]
    L.dg_device_alloc.argtypes = [vp, sz, ctypes.POINTER(vp)]
    L.dg_device_free.argtypes = [vp, vp]
    L.dg_memcpy_h2d.argtypes = [vp, vp, vp, sz]
    L.dg_memcpy_d2h.argtypes = [vp, vp, vp, sz]
    L.dg_synchronize.argtypes = [vp]
    L.dg_host_register.argtypes = [vp, vp, sz]
    L.dg_host_unregister.argtypes = [vp, vp]
    L.dg_last_batch_timings.argtypes = [vp, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(ctypes.c_float), i32]
    L.dg_ctx_set_option.argtypes = [vp, ctypes.c_char_p, ctypes.c_int64]
    L.dg_ctx_get_stat.argtypes = [vp, ctypes.c_char_p]
    L.dg_ctx_get_stat.restype = ctypes.c_int64
    L.dg_last_error.restype = ctypes.c_char_p
    L.dg_sample_align.argtypes = [vp, i32, u8pp, ctypes.POINTER(sz), i32, ctypes.POINTER(i32)]
    L.dg_wds_index.argtypes = [vp, sz, i32, i32, ctypes.c_char_p, vp, ctypes.c_int64, ctypes.POINTER(ctypes.c_int64),
                               vp, sz, ctypes.POINTER(sz), vp, ctypes.c_int64, ctypes.POINTER(ctypes.c_int64)]
    L.dg_wds_key_hash.argtypes = [ctypes.c_char_p, sz]
    L.dg_wds_key_hash.restype = ctypes.c_uint64
    _lib = L
    return L


def last_error() -> str:
    return load().dg_last_error().decode(errors="replace")


def _check(st: int) -> None:
    if st != DG_OK:
        raise DgError(st, last_error())


# ------------------------------------------------------------------ buckets

class BucketTable:
    """dg_bucket_table: ImageTransformConfig::get_ar_aware_transform."""

    def __init__(self, default_image_size: int, downsampling_ratio: int, min_ar: float, max_ar: float,
                 _borrowed: Optional[int] = None):
        L = load()
        self._owned = _borrowed is None
        if _borrowed is not None:
            self._h = ctypes.c_void_p(_borrowed)
        else:
            h = ctypes.c_void_p()
            _check(L.dg_bucket_table_build(default_image_size, downsampling_ratio, min_ar, max_ar,
                                           ctypes.byref(h)))
            self._h = h

    def __del__(self):
        if getattr(self, "_owned", False) and self._h and _lib is not None:
            _lib.dg_bucket_table_free(self._h)

    def __len__(self) -> int:
        return load().dg_bucket_count(self._h)

    def get(self, i: int) -> Tuple[int, int, str]:
        w, h = ctypes.c_uint32(), ctypes.c_uint32()
        key = ctypes.create_string_buffer(32)
        _check(load().dg_bucket_get(self._h, i, ctypes.byref(w), ctypes.byref(h), key, 32))
        return w.value, h.value, key.value.decode()

    def buckets(self) -> List[Tuple[int, int, str]]:
        return [self.get(i) for i in range(len(self))]

    def closest(self, w: int, h: int) -> int:
        return load().dg_closest_bucket(self._h, w, h)

    def find_key(self, key: str) -> int:
        return load().dg_bucket_find_key(self._h, key.encode())


def aspect_ratio_to_str(w: int, h: int) -> str:
    buf = ctypes.create_string_buffer(64)
    _check(load().dg_aspect_ratio_to_str(w, h, buf, 64))
    return buf.value.decode()


def probe(data: bytes) -> Tuple[int, ProbeInfo]:
    info = ProbeInfo()
    st = load().dg_probe(data, len(data), ctypes.byref(info))
    return st, info


def sample_align(table: Optional["BucketTable"], datas: Sequence[bytes], forced_first: int = -1) -> List[int]:
    """dg_sample_align: forced bucket per payload of one sample (reference
    first; worker_wds.rs:68-76).  table None = no image_config."""
    n = len(datas)
    bufs = [ctypes.create_string_buffer(d, len(d)) for d in datas]
    srcs = _as_ptr_array([ctypes.addressof(b) for b in bufs])
    lens = (ctypes.c_size_t * max(1, n))(*[len(d) for d in datas])
    out = (ctypes.c_int32 * max(1, n))()
    _check(load().dg_sample_align(table._h if table is not None else None, n, srcs, lens, forced_first, out))
    return [out[i] for i in range(n)]


class WdsMember(ctypes.Structure):
    _fields_ = [("name_off", ctypes.c_uint64), ("data_off", ctypes.c_uint64), ("data_len", ctypes.c_uint64),
                ("name_len", ctypes.c_uint32), ("pad", ctypes.c_uint32)]


class WdsSample(ctypes.Structure):
    _fields_ = [("first", ctypes.c_uint32), ("count", ctypes.c_uint32)]


def wds_index(tar, rank: int = 0, world_size: int = 1, reference_ext: str = "jpg"):
    """dg_wds_index over a shard in memory (bytes or a uint8 numpy array).
    Returns [[(name, data_off, data_len), ...] per sample]."""
    L = load()
    buf = np.frombuffer(tar, np.uint8) if not isinstance(tar, np.ndarray) else tar
    ptr = buf.ctypes.data
    nm, nn, ns = ctypes.c_int64(), ctypes.c_size_t(), ctypes.c_int64()
    st = L.dg_wds_index(ptr, buf.nbytes, rank, world_size, reference_ext.encode(), None, 0, ctypes.byref(nm), None,
                        0, ctypes.byref(nn), None, 0, ctypes.byref(ns))
    if st not in (DG_OK, DG_ERR_SMALL_BUFFER):
        _check(st)
    mem = (WdsMember * max(1, nm.value))()
    names = ctypes.create_string_buffer(max(1, nn.value))
    sam = (WdsSample * max(1, ns.value))()
    _check(L.dg_wds_index(ptr, buf.nbytes, rank, world_size, reference_ext.encode(), mem, nm.value, ctypes.byref(nm),
                          names, nn.value, ctypes.byref(nn), sam, ns.value, ctypes.byref(ns)))
    raw = names.raw
    out = []
    for s in sam[: ns.value]:
        out.append([(raw[m.name_off:m.name_off + m.name_len].decode("utf-8", "replace"), m.data_off, m.data_len)
                    for m in mem[s.first:s.first + s.count]])
    return out


def wds_key_hash(key: str) -> int:
    b = key.encode()
    return load().dg_wds_key_hash(b, len(b))


# ------------------------------------------------------------------ context

def _as_ptr_array(ptrs: Sequence[int]):
    """Pointer array argument: a uint64 numpy array is passed in place, a
    sequence of ints is converted in one call (no per-element assignment)."""
    if isinstance(ptrs, np.ndarray):
        return _as_array(ctypes.c_void_p, np.uint64, ptrs, ptrs.size)
    return (ctypes.c_void_p * max(1, len(ptrs)))(*ptrs)


def _as_array(ctype, npdtype, vals, n: int):
    """Typed array argument (numpy arrays in place, like _as_ptr_array; a
    read-only or non-contiguous array is copied: from_buffer needs a
    writable buffer)."""
    if isinstance(vals, np.ndarray):
        a = np.require(vals, dtype=npdtype, requirements=["C", "W"])
        if a.size == 0:
            a = np.zeros(1, npdtype)
        return (ctype * a.size).from_buffer(a)
    return (ctype * max(1, n))(*vals)


def meta_status(metas) -> np.ndarray:
    """The status field of every PayloadMeta in a metas array, as int32s (a
    view, no per-element attribute access)."""
    raw = np.frombuffer(metas, dtype=np.uint8).reshape(len(metas), ctypes.sizeof(PayloadMeta))
    off = PayloadMeta.status.offset
    return raw[:, off:off + 4].copy().view(np.int32).reshape(-1)


# Contexts still open at interpreter exit are closed in creation order's
# reverse by an atexit hook, while the HIP runtime and every thread's buffers
# still exist (a context may sit in a reference cycle, or in a module global
# whose __del__ never runs).  DG_NO_ATEXIT_CLOSE=1 leaves them to the
# library's own exit hook (the path a non-Python host takes).
_live: "weakref.WeakValueDictionary[int, Context]" = weakref.WeakValueDictionary()
_live_seq = [0]


def close_all() -> None:
    """Close every context still open, newest first."""
    for k in sorted(_live.keys(), reverse=True):
        c = _live.get(k)
        if c is not None:
            c.close()


def _close_all_at_exit() -> None:
    # dg_ctx_destroy waits for exclusive use of the context.  At interpreter
    # exit only daemon threads are left, and one of them may be inside a long
    # dg_wait / dg_decode_one: then the contexts are left to the
    # library's exit hook, which skips a context that is still in use
    # (try-lock) instead of blocking the exit.
    import threading
    if os.environ.get("DG_NO_ATEXIT_CLOSE") == "1":
        return
    if any(t.is_alive() and t is not threading.current_thread() for t in threading.enumerate()):
        return
    close_all()


atexit.register(_close_all_at_exit)


class Context:
    """dg_ctx: one HIP stream + device arenas on one device (rank -> device)."""

    def __init__(self, device: int = 0, crop_and_resize: bool = False, default_image_size: int = 0,
                 downsampling_ratio: int = 0, min_aspect_ratio: float = 0.0, max_aspect_ratio: float = 0.0,
                 image_to_rgb8: bool = False, pre_encode_images: bool = False, encode_format: int = 0,
                 jpeg_quality: int = 92, decode_semantics: int = 0):
        L = load()
        cfg = ImageConfig(int(crop_and_resize), default_image_size, downsampling_ratio, min_aspect_ratio,
                          max_aspect_ratio, int(pre_encode_images), int(image_to_rgb8), encode_format,
                          jpeg_quality, decode_semantics)
        h = ctypes.c_void_p()
        self._h = None
        _check(L.dg_ctx_create(device, ctypes.byref(cfg), ctypes.byref(h)))
        self._h = h
        _live_seq[0] += 1
        _live[_live_seq[0]] = self
        self.device = device
        self.cfg = cfg
        bt = L.dg_ctx_buckets(h)
        self.buckets = BucketTable(0, 0, 0, 0, _borrowed=bt) if bt else None

    def close(self) -> None:
        h, self._h = getattr(self, "_h", None), None
        if h and _lib is not None:
            _lib.dg_ctx_destroy(h)

    def __del__(self):
        self.close()

    def set_option(self, key: str, value: int) -> None:
        _check(load().dg_ctx_set_option(self._h, key.encode(), int(value)))

    def stat(self, key: str) -> int:
        return load().dg_ctx_get_stat(self._h, key.encode())

    def timings(self) -> dict:
        names = (ctypes.c_char_p * 32)()
        ms = (ctypes.c_float * 32)()
        n = load().dg_last_batch_timings(self._h, names, ms, 32)
        return {names[i].decode(): ms[i] for i in range(n)}

    def output_size(self, data: bytes, forced_bucket: int = -1) -> Tuple[int, int]:
        n = ctypes.c_uint64()
        st = load().dg_output_size(self._h, data, len(data), forced_bucket, ctypes.byref(n))
        return st, n.value

    def sample_align(self, datas: Sequence[bytes], forced_first: int = -1) -> List[int]:
        return sample_align(self.buckets, datas, forced_first)

    # -- host memory in, host memory out (the Rust workers' path)
    def decode_batch(self, datas: Sequence[bytes], forced: Optional[Sequence[int]] = None
                     ) -> List[Tuple[int, Optional[np.ndarray], PayloadMeta]]:
        n = len(datas)
        L = load()
        outs, caps = [], []
        for i, d in enumerate(datas):
            st, nb = self.output_size(d, forced[i] if forced else -1)
            outs.append(np.empty(max(nb, 1), np.uint8))
            caps.append(max(nb, 1))
        # borrowed for the call (dg_submit copies them into pinned staging): no Python-side copy
        bufs = [ctypes.c_char_p(d) for d in datas]
        srcs = _as_ptr_array([ctypes.cast(b, ctypes.c_void_p).value or 0 for b in bufs])
        lens = (ctypes.c_size_t * max(1, n))(*[len(d) for d in datas])
        fb = (ctypes.c_int32 * max(1, n))(*(forced if forced else [-1] * n))
        optrs = _as_ptr_array([o.ctypes.data for o in outs])
        capa = (ctypes.c_uint64 * max(1, n))(*caps)
        metas = (PayloadMeta * max(1, n))()
        ticket = ctypes.c_uint64()
        _check(L.dg_submit(self._h, n, srcs, lens, fb, optrs, capa, metas, ctypes.byref(ticket)))
        _check(L.dg_wait(self._h, ticket.value))
        res = []
        for i in range(n):
            m = metas[i]
            if m.status != DG_OK:
                res.append((m.status, None, m))
                continue
            if m.is_encoded:  # pre_encode_images: the JPEG bytes
                res.append((DG_OK, outs[i][: m.nbytes].copy(), m))
                continue
            c = int(m.nbytes // (m.width * m.height)) if m.width and m.height else 0
            res.append((DG_OK, outs[i][: m.nbytes].reshape(m.height, m.width, c), m))
        return res

    def decode_one(self, data: bytes, forced_bucket: int = -1, out: Optional[np.ndarray] = None):
        """dg_decode_one: one image; concurrent callers (threads) are coalesced
        into shared GPU batches by the library.  `out`: a reused (ideally
        host_register'ed) uint8 buffer of at least output_size bytes.  With
        `out` given the header pass is the library's own: a buffer that turns
        out too small (DG_ERR_SMALL_BUFFER, meta.nbytes = the size needed) is
        replaced and the call made once more."""
        L = load()
        m = PayloadMeta()
        if out is not None and out.nbytes > 0:
            st = L.dg_decode_one(self._h, data, len(data), forced_bucket, out.ctypes.data, out.nbytes,
                                 ctypes.byref(m))
            if st != DG_ERR_SMALL_BUFFER:
                if st != DG_OK:
                    return st, None, m
                c = int(m.nbytes // (m.width * m.height)) if m.width and m.height else 0
                return DG_OK, out[: m.nbytes].reshape(m.height, m.width, c), m
            nb = int(m.nbytes)
        else:
            st, nb = self.output_size(data, forced_bucket)
            if st != DG_OK:
                return st, None, PayloadMeta()
        out = np.empty(max(nb, 1), np.uint8)
        m = PayloadMeta()
        st = L.dg_decode_one(self._h, data, len(data), forced_bucket, out.ctypes.data, max(nb, 1),
                             ctypes.byref(m))
        if st != DG_OK:
            return st, None, m
        c = int(m.nbytes // (m.width * m.height)) if m.width and m.height else 0
        return DG_OK, out[: m.nbytes].reshape(m.height, m.width, c), m

    # -- host bytes in, HBM out (a training loop consumes the tensors where they are)
    def decode_batch_torch(self, datas: Sequence[bytes], forced: Optional[Sequence[int]] = None):
        """Coded bytes go up once (PCIe carries the compressed stream, ~10x
        less than the decoded pixels); outputs are torch uint8 CUDA tensors
        the kernels write directly (no D2H, no host copy).  Returns
        [(status, tensor or None, meta)]; HWC tensors, or 1-D bytes when
        re-encoded."""
        import torch as _t
        n = len(datas)
        fb = list(forced) if forced else [-1] * n
        dev = _t.device("cuda", self.device)
        offs, o = [], 0
        for d in datas:
            offs.append(o)
            o += (len(d) + 16 + 15) // 16 * 16
        host = _t.zeros(max(o, 16), dtype=_t.uint8).pin_memory()
        hv = host.numpy()
        for d, of in zip(datas, offs):
            hv[of:of + len(d)] = np.frombuffer(d, np.uint8)
        dev_in = host.to(dev, non_blocking=False)
        sizes = [self.output_size(d, f)[1] for d, f in zip(datas, fb)]
        outs = [_t.empty(max(nb, 1), dtype=_t.uint8, device=dev) for nb in sizes]
        _t.cuda.current_stream(dev).synchronize()  # inputs resident before the library's streams read them
        hbase, dbase = host.data_ptr(), dev_in.data_ptr()
        ticket, metas = self.submit_device([hbase + of for of in offs], [dbase + of for of in offs],
                                           [len(d) for d in datas], [t.data_ptr() for t in outs],
                                           [max(nb, 1) for nb in sizes], fb)
        self.wait(ticket)
        res = []
        for i in range(n):
            m = metas[i]
            if m.status != DG_OK:
                res.append((m.status, None, m))
            elif m.is_encoded:
                res.append((DG_OK, outs[i][: m.nbytes], m))
            else:
                c = int(m.nbytes // (m.width * m.height)) if m.width and m.height else 0
                res.append((DG_OK, outs[i][: m.nbytes].view(m.height, m.width, c), m))
        del dev_in, host
        return res

    # -- device-resident path (bench): coded bytes already in HBM
    def alloc(self, nbytes: int) -> int:
        p = ctypes.c_void_p()
        _check(load().dg_device_alloc(self._h, nbytes, ctypes.byref(p)))
        return p.value

    def free(self, ptr: int) -> None:
        _check(load().dg_device_free(self._h, ptr))

    def h2d(self, dst: int, src: np.ndarray) -> None:
        _check(load().dg_memcpy_h2d(self._h, dst, src.ctypes.data, src.nbytes))

    def d2h(self, dst: np.ndarray, src: int) -> None:
        _check(load().dg_memcpy_d2h(self._h, dst.ctypes.data, src, dst.nbytes))

    def synchronize(self) -> None:
        _check(load().dg_synchronize(self._h))

    def submit_device(self, h_ptrs, d_ptrs, lens, d_outs, caps, forced=None):
        """Asynchronous device-resident batch; returns (ticket, metas)."""
        n = len(d_ptrs)
        hp = _as_ptr_array(h_ptrs)
        dp = _as_ptr_array(d_ptrs)
        la = _as_array(ctypes.c_size_t, np.uint64, lens, n)
        fb = _as_array(ctypes.c_int32, np.int32, forced if forced is not None else np.full(n, -1, np.int32), n)
        op = _as_ptr_array(d_outs)
        ca = _as_array(ctypes.c_uint64, np.uint64, caps, n)
        metas = (PayloadMeta * max(1, n))()
        ticket = ctypes.c_uint64()
        _check(load().dg_submit_device(self._h, n, hp, dp, la, fb, op, ca, metas, ctypes.byref(ticket)))
        return ticket.value, metas

    def wait(self, ticket: int) -> None:
        _check(load().dg_wait(self._h, ticket))

    def wait_ready(self, ticket: int) -> int:
        """dg_wait_ready: every non-progressive member done; returns how many
        progressive members still run (complete them with wait(ticket))."""
        pend = ctypes.c_int32()
        _check(load().dg_wait_ready(self._h, ticket, ctypes.byref(pend)))
        return pend.value

    def poll(self, ticket: int) -> int:
        return load().dg_poll(self._h, ticket)

    def submit_host(self, datas: Sequence[bytes], outs: Sequence[np.ndarray], forced=None):
        """Asynchronous host-in / host-out batch (dg_submit) into caller-owned
        output arrays (reuse them: with dg_host_register'ed memory the outputs
        arrive by DMA, without staging or page faults).  Returns (ticket,
        metas, keepalive); call wait(ticket) before reading outs or metas."""
        n = len(datas)
        bufs = [ctypes.c_char_p(d) for d in datas]
        srcs = _as_ptr_array([ctypes.cast(b, ctypes.c_void_p).value or 0 for b in bufs])
        lens = (ctypes.c_size_t * max(1, n))(*[len(d) for d in datas])
        fb = (ctypes.c_int32 * max(1, n))(*(forced if forced is not None else [-1] * n))
        optrs = _as_ptr_array([o.ctypes.data for o in outs])
        capa = (ctypes.c_uint64 * max(1, n))(*[o.nbytes for o in outs])
        metas = (PayloadMeta * max(1, n))()
        ticket = ctypes.c_uint64()
        _check(load().dg_submit(self._h, n, srcs, lens, fb, optrs, capa, metas, ctypes.byref(ticket)))
        # keepalive: the output arrays too -- the batch writes them until wait(ticket)
        return ticket.value, metas, (bufs, srcs, lens, fb, optrs, capa, list(outs))

    def host_register(self, arr: np.ndarray) -> None:
        """dg_host_register: page-lock a reused output array (or arena)."""
        _check(load().dg_host_register(self._h, arr.ctypes.data, arr.nbytes))

    def host_unregister(self, arr: np.ndarray) -> None:
        _check(load().dg_host_unregister(self._h, arr.ctypes.data))
