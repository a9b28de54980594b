"""Sample sharding across ranks (one process per GPU, no collectives).

datago never exchanges samples between ranks: each rank decides on its own
which samples it owns, and this module restates those two rules exactly so a
GPU rank feeds its context the same samples the reference rank would.

* file source: contiguous slice, ``get_data_slice_multirank``
  (/root/reference/src/generator_files.rs:24-42);
* WebDataset: ``DefaultHasher`` (SipHash-1-3, keys 0/0) of the member's file
  stem, ``% world_size`` (generator_wds.rs:50-54, 133-148).  Rust's
  ``impl Hash for str`` feeds the UTF-8 bytes followed by one 0xFF byte.

``max_over_ranks`` is the timing reduction bench.py uses (the only
torch.distributed traffic on the path: barriers plus one small all_reduce).
"""
from __future__ import annotations

_M64 = (1 << 64) - 1


def get_data_slice_multirank(quorum: int, rank: int, world_size: int) -> tuple[int, int]:
    """(start, end) of rank's contiguous share of `quorum` samples
    (generator_files.rs:24-42: the first `quorum % world` ranks get one extra)."""
    if not 0 <= rank < world_size:
        raise ValueError("Rank must be less than world size")
    chunk, rem = divmod(quorum, world_size)
    start = rank * (chunk + 1) if rank < rem else rem * (chunk + 1) + (rank - rem) * chunk
    end = (rank + 1) * (chunk + 1) if rank + 1 <= rem else rem * (chunk + 1) + (rank + 1 - rem) * chunk
    return start, end


def _rotl(x: int, b: int) -> int:
    return ((x << b) | (x >> (64 - b))) & _M64


def siphash(data: bytes, k0: int = 0, k1: int = 0, c_rounds: int = 1, d_rounds: int = 3) -> int:
    """SipHash-c-d (Aumasson & Bernstein 2012).  Rust's DefaultHasher is
    SipHash-1-3 with k0 = k1 = 0; c=2,d=4 reproduces the paper's test vector."""
    v0 = k0 ^ 0x736F6D6570736575
    v1 = k1 ^ 0x646F72616E646F6D
    v2 = k0 ^ 0x6C7967656E657261
    v3 = k1 ^ 0x7465646279746573

    def rounds(n):
        nonlocal v0, v1, v2, v3
        for _ in range(n):
            v0 = (v0 + v1) & _M64; v1 = _rotl(v1, 13); v1 ^= v0; v0 = _rotl(v0, 32)
            v2 = (v2 + v3) & _M64; v3 = _rotl(v3, 16); v3 ^= v2
            v0 = (v0 + v3) & _M64; v3 = _rotl(v3, 21); v3 ^= v0
            v2 = (v2 + v1) & _M64; v1 = _rotl(v1, 17); v1 ^= v2; v2 = _rotl(v2, 32)

    n = len(data)
    full = n - n % 8
    for i in range(0, full, 8):
        m = int.from_bytes(data[i:i + 8], "little")
        v3 ^= m
        rounds(c_rounds)
        v0 ^= m
    last = ((n & 0xFF) << 56) | int.from_bytes(data[full:] + b"\0" * (8 - (n - full)), "little")
    v3 ^= last
    rounds(c_rounds)
    v0 ^= last
    v2 ^= 0xFF
    rounds(d_rounds)
    return v0 ^ v1 ^ v2 ^ v3


def wds_hash(key: str) -> int:
    """hash_fn(&str) of generator_wds.rs:50-54 (str bytes + 0xFF terminator)."""
    return siphash(key.encode("utf-8") + b"\xff")


def wds_rank_of(key: str, world_size: int) -> int:
    """Target rank of a WebDataset member with file stem `key` (:133-148);
    world_size <= 1 keeps everything on rank 0."""
    return 0 if world_size <= 1 else wds_hash(key) % world_size


def max_over_ranks(values, world_size: int):
    """Element-wise max of a list of floats over all ranks (gloo/RCCL
    all_reduce; identity when world_size == 1)."""
    import torch
    t = torch.tensor(list(values), dtype=torch.float64)
    if world_size > 1:
        import torch.distributed as dist
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return t.tolist()


def sum_over_ranks(values, world_size: int):
    import torch
    t = torch.tensor(list(values), dtype=torch.float64)
    if world_size > 1:
        import torch.distributed as dist
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return t.tolist()
