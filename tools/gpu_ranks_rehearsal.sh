#!/bin/bash
# Rehearse bench.py's multi-rank path (torch.distributed.run, barrier + max-over-ranks
# timing, one JSON line from rank 0) with two ranks sharing the box's one GPU over gloo
# (RCCL refuses two ranks on one device): prove mode, hot-path mode with the sharded MSM,
# and the standalone MSM replicas.
set -euo pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/ranks
mkdir -p $O
R="python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533"
timeout -k 10 300 $R bench.py --gpus 2 --dist-backend gloo --log-n 16 --lanes 2 --steps 3 --warmup 1 --no-cpu-baseline > $O/prove.log 2>&1
grep '"metric"' $O/prove.log
timeout -k 10 300 $R bench.py --gpus 2 --dist-backend gloo --mode hotpath --shard-msm --log-n 16 --steps 3 --warmup 1 > $O/shard.log 2>&1
grep '"metric"' $O/shard.log
timeout -k 10 300 $R bench.py --gpus 2 --dist-backend gloo --mode msm --log-n 16 --steps 3 --warmup 1 > $O/msm.log 2>&1
grep '"metric"' $O/msm.log
echo done
