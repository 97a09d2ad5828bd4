#!/bin/bash
# Round-3 evidence, part 1: every GPU test, then tools/gpu_profile.sh (default bench under
# --kernel-trace --stats, FETCH / WRITE PMC passes, single-lane breakdowns at 2^20 / 2^16).
set -o pipefail
export TMPDIR=/tmp
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/refresh
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/refresh/pytest.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/refresh/pytest.log; exit 1; }
tail -1 gpurun_out/refresh/pytest.log
bash tools/gpu_profile.sh || exit 1
