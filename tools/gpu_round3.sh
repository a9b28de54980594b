#!/bin/bash
# Round-3 evidence: GPU tests, smoke, 20-step bench, rocprof kernel stats, PMC traffic passes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
STEPS=20 bash tools/gpu_check.sh || exit $?
STEPS=2 bash tools/gpu_pmc.sh || exit $?
