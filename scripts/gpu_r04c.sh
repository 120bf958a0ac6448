mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -m gpu -x -v --timeout 200 --timeout-method thread tests/test_gpu_ops.py -k "sort_pairs or join_table or nin_gemm or nbr" > gpurun_out/pytest_r04c_unit.log 2>&1 || { tail -30 gpurun_out/pytest_r04c_unit.log; exit 1; }
tail -3 gpurun_out/pytest_r04c_unit.log
TAG=r04c STEPS=test bash scripts/gpu_r04.sh || exit 1
TAG=r04c_bnu ROUNDS=2 BENCH_ARGS="--steps 15 --warmup 5 --no-cpu" bash scripts/gpu_ab.sh
