#!/bin/bash
# Round 3, first GPU call: host CPU-share probe, the new GPU tests first (2^20 fixture,
# sharded lanes through the exchange service, large-SRS shards), then the whole -m gpu suite
# and the default bench line. Every step under its own time limit; stop at the first failure.
set -uo pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r03a
mkdir -p $O
{
  echo "nproc $(nproc)"; python3 -c "import os; print('affinity', len(os.sched_getaffinity(0)))"
  cat /sys/fs/cgroup/cpu.max 2>/dev/null || echo "no cpu.max"
  echo "OMP_NUM_THREADS=${OMP_NUM_THREADS:-unset}"; grep -m1 "model name" /proc/cpuinfo
  free -g | head -2
} > $O/host.txt 2>&1
cat $O/host.txt
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 600 --timeout-method thread \
  "tests/test_prover_oracle.py::test_gpu_proof_equals_oracle_fixture_2_20" \
  "tests/test_parallel.py::test_sharded_prover_lanes_exchange_service" \
  "tests/test_parallel.py::test_sharded_prover_three_ranks_large_srs" \
  "tests/test_parallel.py::test_sharded_prover_2_20_equals_fixture" > $O/pytest_new.log 2>&1 \
  || { echo NEW_TESTS_FAILED; tail -60 $O/pytest_new.log; exit 1; }
grep -E "PASSED|FAILED|passed|failed" $O/pytest_new.log | tail -6
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 \
  || { echo TESTS_FAILED; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/bench20.log 2>&1 || { tail -30 $O/bench20.log; exit 1; }
grep '"metric"' $O/bench20.log | cut -c1-300
echo done
