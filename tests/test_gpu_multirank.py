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


def test_two_ranks_through_the_library(tmp_path):
    n, world = 21, 2
    env = dict(os.environ, WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_port()))
    procs = [subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "rank_worker.py"), str(tmp_path), str(n)],
                              env=dict(env, RANK=str(r), LOCAL_RANK=str(r))) for r in range(world)]
    for p in procs:
        assert p.wait(timeout=240) == 0
    got = [np.load(tmp_path / f"rank{r}.npz") for r in range(world)]
    idx = [set(g["indices"].tolist()) for g in got]
    assert idx[0].isdisjoint(idx[1]) and idx[0] | idx[1] == set(range(n))
    assert [len(i) for i in idx] == [11, 10]  # the first n % world ranks take one extra
    datas = synth.mixed_corpus(11, n, 96, 640)
    t = B.ARAwareTransform(512, 16, 0.5, 2.0)
    for g in got:
        assert (g["status"] == 0).all()
        for i in g["indices"].tolist():
            _, dec = O.jpeg_decode(datas[i])
            ref = O.crop_and_resize(dec, *t.target_size(dec.shape[1], dec.shape[0]), O.MODE_FIR)
            assert np.array_equal(g[f"img{i}"], ref), i


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
