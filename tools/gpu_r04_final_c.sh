#!/bin/bash
# Round-4 final check on the final code: the whole -m gpu suite, smoke(), then the rocprof
# evidence job (tools/gpu_profile.sh: default bench under --kernel-trace --stats, PMC traffic
# passes, single-lane proof breakdowns).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/finalc
rm -rf $O; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -n 1 $O/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -n 1 $O/smoke.log
bash tools/gpu_profile.sh
