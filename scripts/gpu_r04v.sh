#!/bin/bash
# Round-4: far rules of the chunk weight gradient (msp_wgrad_far_list + msp_conv_wgrad_far): the wgrad / metadata /
# encoder tests, then the per-shape bench (the level of the second batch whose tiles exceed the cap now stays on
# the chunk form) and two default bench lines.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_encoders.py -k "wgrad or chunk or prefetch or graph or metadata or parity" > gpurun_out/pytest_r04v.log 2>&1 || { tail -30 gpurun_out/pytest_r04v.log; exit 1; }
tail -2 gpurun_out/pytest_r04v.log
MI3DSPARSE_KIND_SHAPES=1 timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu > gpurun_out/bench_r04v_shapes.log 2>&1 || exit 1
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/bench_r04v_$i.log 2>&1 || exit 1
  grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_r04v_$i.log
done
