set -eo pipefail
mkdir -p gpurun_out/r06q
for rep in 1 2; do for q in 24 28 32; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --hw-queues $q > gpurun_out/r06q/q${q}_$rep.json 2> gpurun_out/r06q/q${q}_$rep.err
done; done
