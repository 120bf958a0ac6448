# N-rank checks on a one-GPU box: the DDP / graph-DP GPU tests (gloo, two ranks on cuda:0) and a two-rank bench
# rehearsal of the graph path (gloo, shared device).  Usage: bash scripts/gpu_dp.sh TAG
set -o pipefail
TAG=${1:-dp}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_ddp.py -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_$TAG.log 2>&1; rc=$?; tail -5 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
BENCH_BACKEND=gloo BENCH_SHARE_DEVICE=1 timeout -k 10 500 python bench.py --gpus 2 --steps 6 --warmup 2 --no-cpu \
  > gpurun_out/bench_$TAG.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/bench_$TAG.log | tail -c 1500; exit $rc
