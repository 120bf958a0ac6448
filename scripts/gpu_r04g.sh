#!/bin/bash
# Round-4 host-side profile of the C2 and C3 steps (scripts/host_profile.py) and the C2 preset bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
PRESET=c2 STEPS=5 TOP=45 timeout -k 10 300 python -u scripts/host_profile.py > gpurun_out/host_r04g_c2.log 2>&1 || exit 1
head -8 gpurun_out/host_r04g_c2.log
timeout -k 10 300 python -u bench.py --preset c2 --steps 20 --warmup 5 --no-cpu > gpurun_out/bench_r04g_c2.log 2>&1 || exit 1
BENCH_HOST_TIMING=1 timeout -k 10 300 python -u bench.py --preset c2 --steps 20 --warmup 5 --no-cpu > gpurun_out/bench_r04g_c2_host.log 2>&1 || exit 1
grep "graph loop host" gpurun_out/bench_r04g_c2_host.log; grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_r04g_c2.log
BENCH_HOST_TIMING=1 timeout -k 10 300 python -u bench.py --steps 15 --warmup 5 --no-cpu > gpurun_out/bench_r04g_c3_host.log 2>&1 || exit 1
grep "graph loop host\|device idle" gpurun_out/bench_r04g_c3_host.log | cut -c1-400; grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_r04g_c3_host.log
