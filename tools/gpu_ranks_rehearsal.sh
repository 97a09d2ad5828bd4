#!/bin/bash
# Rehearse bench.py's multi-rank paths with two ranks sharing the box's one GPU over gloo
# (RCCL refuses two ranks on one device); bench.py --gpus 2 launches the ranks itself
# (torch.distributed.run child process): proof batches, the sharded full prover
# (configs[4] form), the sharded-MSM hot path and the standalone MSM replicas.
set -euo pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/ranks
mkdir -p $O
G="--gpus 2 --dist-backend gloo"
timeout -k 10 300 python3 bench.py $G --log-n 16 --lanes 2 --steps 3 --warmup 1 --no-cpu-baseline > $O/prove.log 2>&1
grep '"metric"' $O/prove.log
timeout -k 10 300 python3 bench.py $G --shard-msm --log-n 16 --lanes 2 --steps 3 --warmup 1 --no-cpu-baseline > $O/prove_shard.log 2>&1
grep '"metric"' $O/prove_shard.log
timeout -k 10 300 python3 bench.py $G --mode hotpath --shard-msm --log-n 16 --steps 3 --warmup 1 > $O/hotpath_shard.log 2>&1
grep '"metric"' $O/hotpath_shard.log
timeout -k 10 300 python3 bench.py $G --mode msm --log-n 16 --steps 3 --warmup 1 > $O/msm.log 2>&1
grep '"metric"' $O/msm.log
echo done
