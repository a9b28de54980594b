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
