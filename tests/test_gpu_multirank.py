"""Multi-rank runs through the library.

One process per rank, started the way torchrun starts them (environment set
before the process begins; the parent never hands a GPU context across).
On a one-GPU box the ranks share device 0.  Checks: the ranks' slices
(get_data_slice_multirank, generator_files.rs:24-42) are disjoint and cover
the stream, every output is bit-exact against the oracle, and `bench.py
--gpus 2` (no torchrun) starts two ranks itself and reports n_gpus 2.
"""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from datago_amd import synth
from oracle import buckets as B
from oracle import oracle as O

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run_ranks(tmp_path, n, world, size, ratio):
    env = dict(os.environ, WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_port()))
    procs = [subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "rank_worker.py"), str(tmp_path), str(n),
                               str(size), str(ratio)],
                              env=dict(env, RANK=str(r), LOCAL_RANK=str(r))) for r in range(world)]
    try:
        for p in procs:
            assert p.wait(timeout=300) == 0
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    return [np.load(tmp_path / f"rank{r}.npz") for r in range(world)]


def _check_ranks(got, n, world, size, ratio):
    idx = [set(g["indices"].tolist()) for g in got]
    for a in range(world):
        for b in range(a + 1, world):
            assert idx[a].isdisjoint(idx[b])
    assert set().union(*idx) == set(range(n))
    base, extra = divmod(n, world)  # get_data_slice_multirank: the first n % world ranks take one extra
    assert [len(i) for i in idx] == [base + (r < extra) for r in range(world)]
    datas = synth.mixed_corpus(11, n, 96, 640)
    t = B.ARAwareTransform(size, ratio, 0.5, 2.0)
    for g in got:
        assert (g["status"] == 0).all()
        for i in g["indices"].tolist():
            _, dec = O.jpeg_decode(datas[i])
            ref = O.crop_and_resize(dec, *t.target_size(dec.shape[1], dec.shape[0]), O.MODE_FIR)
            assert np.array_equal(g[f"img{i}"], ref), i


def test_two_ranks_through_the_library(tmp_path):
    _check_ranks(_run_ranks(tmp_path, 21, 2, 512, 16), 21, 2, 512, 16)


def test_eight_ranks_configs3_through_the_library(tmp_path):
    """configs[3]'s world_size 8 (rank r takes get_data_slice_multirank(N, r, 8),
    generator_files.rs:24-42,75-80) with its 1024/32 buckets: eight rank
    processes, each with its own context (all on device 0 of a one-GPU box),
    started before any GPU call as torchrun starts them.  The slices are
    disjoint, cover the stream (43 = 8 x 5 + 3: ranks 0-2 take one extra) and
    every output is bit-exact against the oracle."""
    _check_ranks(_run_ranks(tmp_path, 43, 8, 1024, 32), 43, 8, 1024, 32)


def test_bench_gpus_flag_launches_ranks(tmp_path):
    out = tmp_path / "b.json"
    env = dict(os.environ, DATAGO_CORPUS_CACHE=str(tmp_path / "cache"))
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
                        "--batch", "8", "--pool", "24", "--samples", "64", "--short-max", "512", "--no-cpu-baseline",
                        "--e2e-steps", "0", "--serial-steps", "0", "--out", str(out)], env=env, timeout=400,
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads(out.read_text())
    assert line["n_gpus"] == 2 and len(line["ms_per_step_per_rank"]) == 2
    assert line["value"] > 0 and line["scaling"] == "weak"
