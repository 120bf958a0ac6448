#!/bin/bash
# Round-4: the two-launch radix-sort passes -- sort and metadata tests, then an interleaved A/B against the
# previous build (lib/libmi3dsparse_exp.so = the four-launch passes) with the host timing of the graph loop.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_encoders.py -k "sort or prefetch or graph or metadata or input or fused" > gpurun_out/pytest_r04j.log 2>&1 || { tail -30 gpurun_out/pytest_r04j.log; exit 1; }
tail -2 gpurun_out/pytest_r04j.log
TAG=r04j_sort ROUNDS=3 BENCH_ARGS="--steps 20 --warmup 5 --no-cpu" B_ENV="BENCH_HOST_TIMING=0" bash scripts/gpu_ab.sh || exit 1
for v in A B; do
  lib=""; [ $v = B ] && lib="MI3DSPARSE_LIB=$GRAFT_REPO_ROOT/3d-weakly-supervised-semantic-segmentation_amd/lib/libmi3dsparse_exp.so"
  env $lib BENCH_HOST_TIMING=1 timeout -k 10 300 python -u bench.py --steps 15 --warmup 5 --no-cpu > gpurun_out/bench_r04j_host_$v.log 2>&1 || exit 1
  echo "$v"; grep "graph loop host\|device idle" gpurun_out/bench_r04j_host_$v.log | cut -c1-300
done
