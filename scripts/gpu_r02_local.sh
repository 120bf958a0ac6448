set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread ${TESTS:-tests/test_gpu_ops.py tests/test_gpu_encoders.py tests/test_gpu_fullsize.py tests/test_gpu_golden.py} -m gpu > gpurun_out/pytest_local.log 2>&1 \
 && echo tests ok \
 && timeout -k 10 600 python bench.py --steps 20 --warmup 5 --no-cpu ${BENCH_ARGS} > gpurun_out/bench_local.log 2>&1 && echo bench ok
rc=$?
tail -5 gpurun_out/pytest_local.log; tail -c 400 gpurun_out/bench_local.log
exit $rc
