set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_abi.py tests/test_gpu_heads.py tests/test_gpu_fullsize.py -m gpu > gpurun_out/pytest_new.log 2>&1 \
 && echo tests ok \
 && BENCH_BACKEND=gloo BENCH_SHARE_DEVICE=1 timeout -k 10 300 python bench.py --gpus 2 --steps 3 --warmup 1 --batch 2 > gpurun_out/bench_n2.log 2>&1 \
 && echo n2 ok
rc=$?
tail -25 gpurun_out/pytest_new.log; tail -c 600 gpurun_out/bench_n2.log
exit $rc
