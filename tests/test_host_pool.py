"""HostPool (datago_amd/csrc/host/host_pool.h), the planning workers of
dg_submit*: every index runs exactly once per job, jobs from several threads
serialise, and the pool shuts down cleanly.  Compiled with g++ on the host."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SRC = r"""
#include <cstdio>
#include <vector>
#include "host_pool.h"
int main() {
  for (int threads : {1, 2, 4, 7}) {
    dg::HostPool pool(threads);
    for (int n : {0, 1, 31, 32, 33, 1000, 4097}) {
      for (int grain : {1, 32}) {
        std::vector<int> hit(n, 0);
        pool.run(n, grain, [&](int i) { hit[i]++; });
        for (int i = 0; i < n; i++)
          if (hit[i] != 1) { printf("FAIL t=%d n=%d g=%d i=%d hit=%d\n", threads, n, grain, i, hit[i]); return 1; }
      }
    }
    // concurrent callers: jobs serialise, each still complete
    std::vector<std::thread> cs;
    std::atomic<int> bad{0};
    for (int c = 0; c < 4; c++)
      cs.emplace_back([&] {
        for (int r = 0; r < 50; r++) {
          std::vector<int> hit(300, 0);
          pool.run(300, 8, [&](int i) { hit[i]++; });
          for (int v : hit) bad += v != 1;
        }
      });
    for (auto &t : cs) t.join();
    if (bad) { printf("FAIL concurrent t=%d\n", threads); return 1; }
  }
  printf("OK\n");
  return 0;
}
"""


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_host_pool(tmp_path):
    src = tmp_path / "t.cpp"
    src.write_text(SRC)
    exe = tmp_path / "t"
    subprocess.run(["g++", "-std=c++17", "-O1", "-pthread", "-I", os.path.join(ROOT, "datago_amd/csrc/host"),
                    str(src), "-o", str(exe)], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0 and r.stdout.strip() == "OK", r.stdout + r.stderr
