#!/bin/bash
# Round-4: batched count reads in the metadata replay (metadata._Deferred), the two-launch radix-sort passes, and
# conv_x6s with one offset list shared by both row halves (lib/libmi3dsparse_exp.so built -DMSP_SHARED_LISTS=1).
# Tests first (sort, prefetch / graph / metadata), then the host timing of the graph loop with and without the
# batched reads, an interleaved A/B of them (B = MSP_DEFER_READS=0), and kbench of the tile-local convolution.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=$GRAFT_REPO_ROOT/3d-weakly-supervised-semantic-segmentation_amd/lib
timeout -k 10 400 python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_encoders.py -k "sort or prefetch or graph or metadata or input or fused" > gpurun_out/pytest_r04k.log 2>&1 || { tail -30 gpurun_out/pytest_r04k.log; exit 1; }
tail -2 gpurun_out/pytest_r04k.log
for v in A B; do
  envs="BENCH_HOST_TIMING=1"; [ $v = B ] && envs="$envs MSP_DEFER_READS=0"
  env $envs timeout -k 10 300 python -u bench.py --steps 15 --warmup 5 --no-cpu > gpurun_out/bench_r04k_host_$v.log 2>&1 || exit 1
  echo "$v"; grep "graph loop host\|device idle" gpurun_out/bench_r04k_host_$v.log | cut -c1-300
done
TAG=r04k_defer ROUNDS=3 B_LIB=0 BENCH_ARGS="--steps 20 --warmup 5 --no-cpu" B_ENV="MSP_DEFER_READS=0" bash scripts/gpu_ab.sh || exit 1
for i in 1 2; do
  for v in A B; do
    lib=""; [ $v = B ] && lib="MI3DSPARSE_LIB=$L/libmi3dsparse_exp.so"
    env $lib LEVELS=1,2,3 PASSES=fwd,bwd FORMS=local N=20 timeout -k 10 300 python -u scripts/kbench.py > gpurun_out/kb_r04k_$v$i.log 2>&1 || exit 1
  done
done
grep -h "local" gpurun_out/kb_r04k_A1.log gpurun_out/kb_r04k_B1.log | head -30
