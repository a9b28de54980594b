"""Process exit with live contexts (a bench run under
rocprofv3 printed its line and then died in __cxa_finalize).

tests/exit_worker.py leaves planning workers, coalesced dg_decode_one state,
an open progressive aggregate and an unwaited device batch behind, held by
reference cycles, and returns from main.  Both ways out must end with rc 0:
the Python close-all (`_lib` registers it with atexit) and the library's own
exit hook alone (DG_NO_ATEXIT_CLOSE, what a Rust host that never drops its
stage relies on)."""
import os
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("mode", ["atexit", "raw"])
def test_exit_with_live_contexts(mode):
    r = subprocess.run([sys.executable, os.path.join(HERE, "exit_worker.py"), mode], capture_output=True,
                       text=True, timeout=240)
    assert "EXIT-WORKER-OK" in r.stdout, r.stdout[-2000:] + r.stderr[-4000:]
    assert r.returncode == 0, f"rc {r.returncode}\n{r.stderr[-4000:]}"
