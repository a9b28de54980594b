"""Rank sharding: the file-source slice and the WebDataset
hash restated in datago_amd/sharding.py, plus a world_size-2 gloo run of the
exact reduction bench.py uses."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from datago_amd.sharding import (get_data_slice_multirank, max_over_ranks, siphash, sum_over_ranks,
                                 wds_hash, wds_rank_of)


def test_reference_known_answers():
    # generator_files.rs:191-232 (test_get_data_slice_multirank)
    cases = [((10, 0, 2), (0, 5)), ((10, 1, 2), (5, 10)), ((11, 0, 2), (0, 6)), ((11, 1, 2), (6, 11)),
             ((13, 0, 3), (0, 5)), ((13, 1, 3), (5, 9)), ((13, 2, 3), (9, 13)), ((10, 0, 1), (0, 10)),
             ((0, 0, 1), (0, 0))]
    for args, want in cases:
        assert get_data_slice_multirank(*args) == want


def test_rank_out_of_range_raises():
    # the reference asserts (generator_files.rs:25)
    with pytest.raises(ValueError):
        get_data_slice_multirank(10, 2, 2)


@pytest.mark.parametrize("world", [1, 2, 3, 4, 7, 8])
@pytest.mark.parametrize("quorum", [0, 1, 7, 8, 100, 1001])
def test_slices_partition(world, quorum):
    prev = 0
    for r in range(world):
        s, e = get_data_slice_multirank(quorum, r, world)
        assert s == prev and e >= s and e - s in (quorum // world, quorum // world + 1)
        prev = e
    assert prev == quorum


def test_siphash_paper_vector():
    # Aumasson & Bernstein, SipHash paper appendix A: SipHash-2-4, key 00..0f, msg 00..0e
    k = bytes(range(16))
    k0, k1 = int.from_bytes(k[:8], "little"), int.from_bytes(k[8:], "little")
    assert siphash(bytes(range(15)), k0, k1, 2, 4) == 0xA129CA6149BE45E5


def test_wds_hash_is_str_hash_with_terminator():
    # impl Hash for str: bytes then 0xFF; DefaultHasher = SipHash-1-3(0, 0)
    assert wds_hash("sample_000") == siphash(b"sample_000\xff", 0, 0, 1, 3)
    assert wds_rank_of("anything", 1) == 0
    owners = [wds_rank_of(f"{i:08d}", 8) for i in range(4000)]
    counts = [owners.count(r) for r in range(8)]
    assert min(counts) > 400  # a hash, roughly uniform over ranks


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, n, keys, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        s, e = get_data_slice_multirank(n, rank, world)
        mine = [i for i in range(s, e)]
        wds_mine = [k for k in keys if wds_rank_of(k, world) == rank]
        got = [None] * world
        dist.all_gather_object(got, (mine, wds_mine))
        # the bench reduction: max of times, sum of pixels
        mx = max_over_ranks([float(rank + 1), -float(rank)], world)
        sm = sum_over_ranks([float(e - s)], world)
        dist.barrier()
        if rank == 0:
            q.put((got, mx, sm))
    finally:
        dist.destroy_process_group()


def test_two_rank_gloo_sharding():
    world, n = 2, 1001
    keys = [f"shard{i // 100}_{i:06d}" for i in range(500)]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, keys, q)) for r in range(world)]
    for p in procs:
        p.start()
    got, mx, sm = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    files = [set(g[0]) for g in got]
    assert files[0].isdisjoint(files[1]) and files[0] | files[1] == set(range(n))
    wds = [set(g[1]) for g in got]
    assert wds[0].isdisjoint(wds[1]) and wds[0] | wds[1] == set(keys)
    assert mx == [2.0, 0.0]
    assert sm == [float(n)]
