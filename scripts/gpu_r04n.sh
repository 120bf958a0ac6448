#!/bin/bash
# Round-4: the metadata prefetch on a worker thread beside the capture (bench.py --prefetch-thread 1).  GIL probe,
# prefetch tests, host timing of both loops, then an interleaved A/B (B = --prefetch-thread 1).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 120 python -u scripts/gil_probe.py > gpurun_out/gil_probe_r04n.log 2>&1 || { cat gpurun_out/gil_probe_r04n.log; exit 1; }
cat gpurun_out/gil_probe_r04n.log
timeout -k 10 400 python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread tests/test_gpu_encoders.py -k "prefetch or graph or metadata" > gpurun_out/pytest_r04n.log 2>&1 || { tail -30 gpurun_out/pytest_r04n.log; exit 1; }
tail -2 gpurun_out/pytest_r04n.log
for v in A B; do
  extra=""; [ $v = B ] && extra="--prefetch-thread 1"
  BENCH_HOST_TIMING=1 timeout -k 10 300 python -u bench.py --steps 15 --warmup 5 --no-cpu $extra > gpurun_out/bench_r04n_host_$v.log 2>&1 || { tail -20 gpurun_out/bench_r04n_host_$v.log; exit 1; }
  echo "$v"; grep "graph loop host\|device idle" gpurun_out/bench_r04n_host_$v.log | cut -c1-300
done
TAG=r04n_thread ROUNDS=3 B_LIB=0 BENCH_ARGS="--steps 20 --warmup 5 --no-cpu" B_ARGS="--prefetch-thread 1" bash scripts/gpu_ab.sh || exit 1
