"""WebDataset shard indexing (dg_wds_index, host C++) against a Python
restatement of pull_tarballs (generator_wds.rs:56-204): tar walk, sample key
= Path::file_stem, SipHash-1-3 rank filter, consecutive grouping,
reference extension first."""
import io
import pathlib
import tarfile

import pytest

from datago_amd import _lib as L
from datago_amd import sharding, synth


def _tar(entries, fmt):
    buf = io.BytesIO()
    with tarfile.open(fileobj=buf, mode="w", format=fmt) as tf:
        for name, data in entries:
            if data is None:
                ti = tarfile.TarInfo(name)
                ti.type = tarfile.DIRTYPE
                tf.addfile(ti)
                continue
            ti = tarfile.TarInfo(name)
            ti.size = len(data)
            tf.addfile(ti, io.BytesIO(data))
    return buf.getvalue()


def _reference(tar: bytes, rank, world, ref_ext):
    out, cur, key = [], [], None
    with tarfile.open(fileobj=io.BytesIO(tar)) as tf:
        for m in tf.getmembers():
            if not m.isfile():
                continue
            k = pathlib.PurePosixPath(m.name).stem
            if world > 1 and sharding.siphash(k.encode() + b"\xff") % world != rank:
                continue
            if key is not None and k != key and cur:
                out.append(cur)
                cur = []
            key = k
            cur.append((m.name, m.offset_data, m.size))
    if cur:
        out.append(cur)
    return [[x for x in s if x[0].endswith(ref_ext)] + [x for x in s if not x[0].endswith(ref_ext)] for s in out]


ENTRIES = [("a.cls", b"1"), ("a.jpg", b"JPG-A"), ("b.jpg", b"JPG-B"), ("b.png", b"PNG-B"), ("b.txt", b"t"),
           ("dir", None), ("dir/c.jpg", b"C"), ("x" * 150 + ".jpg", b"LONG"), ("x" * 150 + ".cls", b"7"),
           ("d.e.jpg", b"DE"), (".hidden", b"H"), ("e.jpg", b"")]


@pytest.mark.parametrize("fmt", [tarfile.GNU_FORMAT, tarfile.PAX_FORMAT, tarfile.USTAR_FORMAT])
@pytest.mark.parametrize("world", [1, 2, 3])
def test_index_matches_restatement(fmt, world):
    entries = ENTRIES if fmt != tarfile.USTAR_FORMAT else [e for e in ENTRIES if len(e[0]) < 100]
    tar = _tar(entries, fmt)
    seen = []
    for rank in range(world):
        got = L.wds_index(tar, rank, world, "jpg")
        assert got == _reference(tar, rank, world, "jpg")
        for s in got:
            for name, off, n in s:
                assert tar[off:off + n] == dict(entries)[name]
                seen.append(name)
    assert sorted(seen) == sorted(n for n, d in entries if d is not None)  # disjoint, complete


def test_key_hash_matches_siphash_restatement():
    for key in ["", "a", "n00000001", "x" * 100, "clé"]:
        assert L.wds_key_hash(key) == sharding.siphash(key.encode() + b"\xff")


def test_synthetic_imagenet_shard():
    tar = synth.make_wds_shard(3, 20)
    samples = L.wds_index(tar, 0, 1, "jpg")
    assert len(samples) == 20 and all(len(s) == 2 and s[0][0].endswith(".jpg") for s in samples)
    for s in samples:
        name, off, n = s[0]
        assert tar[off:off + 2] == b"\xff\xd8"


def _raw_header(name: bytes, size_field: bytes, typeflag: bytes) -> bytes:
    """One 512-byte tar header with a caller-chosen 12-byte size field and a
    valid checksum (so only the size/record logic can reject it)."""
    h = bytearray(512)
    h[0:len(name)] = name
    h[100:108] = b"0000644\0"
    h[124:136] = size_field
    h[136:148] = b"00000000000\0"
    h[156:157] = typeflag
    h[257:263] = b"ustar\0"
    h[263:265] = b"00"
    h[148:156] = b" " * 8
    h[148:156] = b"%06o\0 " % sum(h)
    return bytes(h)


def _status(tar: bytes) -> int:
    import ctypes
    import numpy as np
    lib = L.load()
    buf = np.frombuffer(tar, np.uint8)
    nm, ns, nn = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_size_t()
    return lib.dg_wds_index(buf.ctypes.data, buf.nbytes, 0, 1, b"jpg", None, 0, ctypes.byref(nm), None, 0,
                            ctypes.byref(nn), None, 0, ctypes.byref(ns))


@pytest.mark.parametrize("size_field", [
    b"\x80" + b"\xff" * 11,                      # base-256, ~2^88: does not fit 64 bits
    b"\x80\x00\x00\x00" + b"\xff" * 7 + b"\x00",  # base-256 2^64-256: data + size would wrap
    b"\xff" * 12,                                # base-256 negative
    b"77777777777\0",                            # octal 8 GiB, past the buffer
])
def test_hostile_size_field_is_corrupt(size_field):
    tar = _raw_header(b"a.jpg", size_field, b"0") + b"\0" * 2048
    assert _status(tar) == L.DG_ERR_CORRUPT


def test_truncated_long_name_is_corrupt():
    # GNU 'L' entry claiming 4 KiB of name where the buffer ends after 512 bytes
    tar = _raw_header(b"././@LongLink", b"%011o\0" % 4096, b"L") + b"x" * 512
    assert _status(tar) == L.DG_ERR_CORRUPT


@pytest.mark.parametrize("record", [b"2 x", b"3 ab", b"1 ", b"9999999999999999999999 path=a"])
def test_malformed_pax_record_does_not_abort(record):
    body = record + b"\0" * (512 - len(record))
    tar = (_raw_header(b"PaxHeader", b"%011o\0" % len(record), b"x") + body +
           _raw_header(b"a.jpg", b"%011o\0" % 3, b"0") + b"JPG" + b"\0" * 509 + b"\0" * 1024)
    assert L.wds_index(tar, 0, 1, "jpg") == [[("a.jpg", 1536, 3)]]
