set -eo pipefail
python tools/recipes.py ab --out gpurun_out/r06d_ruf --reps 3 --lib base=libplk.so --lib ruf=libplk-ruf.so --env PLK_LIB_ANY_SRC=1 \
  --tests "tests/test_opening_gpu.py tests/test_prover_gpu.py" \
  --args "--log-n 12 --steps 40" --args "--log-n 13 --steps 30" --args "--log-n 14 --steps 20" --limit 1100
python tools/recipes.py ab --out gpurun_out/r06d_c12 --reps 2 --venv c8=PLK_MSM_C=8 --venv c9=PLK_MSM_C=9 --venv c10=PLK_MSM_C=10 \
  --args "--log-n 12 --steps 40" --limit 600
python tools/recipes.py ab --out gpurun_out/r06d_c13 --reps 2 --venv c10=PLK_MSM_C=10 --venv c11=PLK_MSM_C=11 --venv c12=PLK_MSM_C=12 \
  --args "--log-n 13 --steps 30" --limit 600
