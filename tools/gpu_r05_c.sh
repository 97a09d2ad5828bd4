#!/bin/bash
# Round 5 (c): balanced MSM windows (srs.hip: the top c W - 255 windows c - 1 bits, digits x 2,
# instead of one short top window with digits x 2^top_shift) and finer coarse bins for bucket-
# range parts: the whole -m gpu suite, then interleaved A/B against the previous build
# (libplk-prev.so) on lone MSMs, proofs at 2^12 / 2^16 / 2^20 and the 8-part split MSM, and a
# kernel trace of the 8-part run; the pipelined lone NTT pass (k_ntt_pipe, LDS-DMA) against
# k_ntt_pass (PLK_NTT_PIPE=0) at 2^20 and 2^23.
set -o pipefail
mkdir -p gpurun_out/r05c
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r05c/tests.log 2>&1 || { tail -n 40 gpurun_out/r05c/tests.log; exit 1; }
tail -n 1 gpurun_out/r05c/tests.log
timeout -k 10 1000 python -u tools/ab.py --out gpurun_out/r05c/ab.jsonl --reps 2 \
  --lib prev=libplk-prev.so --lib new=libplk.so \
  --args "--mode msm --log-n 20 --steps 30" --args "--mode msm --log-n 20 --steps 10 --bucket-parts 8" \
  --args "--log-n 20 --steps 6" --args "--log-n 16 --steps 10" --args "--log-n 12 --steps 30" || exit 1
timeout -k 10 600 python -u tools/ab.py --out gpurun_out/r05c/ntt_ab.jsonl --reps 2 \
  --venv pipe=PLK_NTT_PIPE=1 --venv nopipe=PLK_NTT_PIPE=0 \
  --args "--mode ntt --log-n 20 --steps 50" --args "--mode ntt --log-n 23 --steps 10" || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05c/prof_parts8 -o run -- \
  python bench.py --mode msm --log-n 20 --steps 10 --warmup 2 --no-cpu-baseline --bucket-parts 8 \
  > gpurun_out/r05c/parts8.json 2> gpurun_out/r05c/parts8.err || { tail -n 20 gpurun_out/r05c/parts8.err; exit 1; }
python tools/rocpd_summary.py gpurun_out/r05c/prof_parts8/run_results.db --after k_double_c --window 12 | tail -n 14
