#!/bin/bash
# Round-4 closing checks on the final tree: smoke, the prefetch / graph / metadata / DDP GPU tests, and a two-rank
# rehearsal of bench.py's N-rank path (two ranks sharing the one GPU over gloo).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.add_path(); g.smoke()" > gpurun_out/smoke_r04z.log 2>&1 || { cat gpurun_out/smoke_r04z.log; exit 1; }
tail -1 gpurun_out/smoke_r04z.log
timeout -k 10 700 python -u -m pytest -m gpu -x -v --timeout 600 --timeout-method thread tests/test_gpu_encoders.py tests/test_gpu_ddp.py -k "prefetch or graph or metadata or ddp or dp or rccl" > gpurun_out/pytest_r04z.log 2>&1 || { tail -30 gpurun_out/pytest_r04z.log; exit 1; }
tail -2 gpurun_out/pytest_r04z.log
BENCH_BACKEND=gloo BENCH_SHARE_DEVICE=1 timeout -k 10 600 python -u bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu > gpurun_out/bench_r04z_n2_gloo.log 2>&1 || { tail -30 gpurun_out/bench_r04z_n2_gloo.log; exit 1; }
grep '^{"metric"' gpurun_out/bench_r04z_n2_gloo.log | cut -c1-300
