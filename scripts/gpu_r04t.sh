#!/bin/bash
# Round-4: the capture's host phases (begin / body / end) and a private pool per graph, with the replay idle.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for v in A B; do
  envs="BENCH_HOST_TIMING=1"; [ $v = B ] && envs="$envs BENCH_GRAPH_PRIVATE_POOL=1"
  env $envs timeout -k 10 300 python -u bench.py --steps 15 --warmup 5 --no-cpu > gpurun_out/bench_r04t_host_$v.log 2>&1 || { tail -20 gpurun_out/bench_r04t_host_$v.log; exit 1; }
  echo "$v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_r04t_host_$v.log)"; grep "graph loop host\|device idle\|capture host\|count reads" gpurun_out/bench_r04t_host_$v.log | cut -c1-200
done
MI3DSPARSE_KIND_SHAPES=1 timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu > gpurun_out/bench_r04t_shapes.log 2>&1 || exit 1
