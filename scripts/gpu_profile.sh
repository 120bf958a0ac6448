#!/bin/bash
# rocprofv3 kernel trace + stats of the bench (STEPS timed steps, graph mode as the driver runs it): the stats
# summary, device idle gaps and the per-step kernel list (scripts/step_kernels.py) under gpurun_out/.
set -o pipefail
TAG=${TAG:-r03} STEPS=${BENCH_STEPS:-10} bash scripts/profile.sh && \
  python3 scripts/prof_summary.py $(find gpurun_out/prof_${TAG} -name "*kernel_stats.csv" | head -1) 45 > gpurun_out/kernel_stats_${TAG}_summary.txt && \
  python3 scripts/trace_gaps.py $(find gpurun_out/prof_${TAG} -name "*kernel_trace.csv" | head -1) > gpurun_out/gaps_${TAG}.txt && \
  python3 scripts/step_kernels.py $(find gpurun_out/prof_${TAG} -name "*kernel_trace.csv" | head -1) > gpurun_out/step_kernels_${TAG}.txt && \
  python3 scripts/step_gaps.py $(find gpurun_out/prof_${TAG} -name "*kernel_trace.csv" | head -1) > gpurun_out/step_gaps_${TAG}.txt && \
  python3 scripts/kernel_by_grid.py $(find gpurun_out/prof_${TAG} -name "*kernel_trace.csv" | head -1) bn_ conv_x6 wgrad_x6 split_cols \
    > gpurun_out/kernel_by_grid_${TAG}.txt
rc=$?
cat gpurun_out/step_kernels_${TAG}.txt 2>/dev/null | head -60
exit $rc
