#!/bin/bash
# One GPU call: the -m gpu suite, then the default bench line (2^20) and the 2^16 line.
# Every step under its own time limit; the chain stops at the first failure.
set -euo pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/check
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/bench20.log 2>&1 || { tail -30 $O/bench20.log; exit 1; }
grep '"metric"' $O/bench20.log | cut -c1-400
timeout -k 10 300 python3 -u bench.py --log-n 16 --steps 20 --warmup 3 --no-cpu-baseline > $O/bench16.log 2>&1 || { tail -30 $O/bench16.log; exit 1; }
grep '"metric"' $O/bench16.log | cut -c1-400
echo done
