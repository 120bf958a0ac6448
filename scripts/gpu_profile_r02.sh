# rocprofv3 kernel trace + stats of the bench (5 timed steps), its summary and the device idle gaps.
set -o pipefail
TAG=${TAG:-r02} STEPS=${STEPS:-5} bash scripts/profile.sh && \
  python3 scripts/prof_summary.py $(find gpurun_out/prof_${TAG:-r02} -name "*kernel_stats.csv" | head -1) 45 > gpurun_out/kernel_stats_${TAG:-r02}_summary.txt && \
  python3 scripts/trace_gaps.py $(find gpurun_out/prof_${TAG:-r02} -name "*kernel_trace.csv" | head -1) > gpurun_out/gaps_${TAG:-r02}.txt
rc=$?
cat gpurun_out/kernel_stats_${TAG:-r02}_summary.txt gpurun_out/gaps_${TAG:-r02}.txt 2>/dev/null | head -70
exit $rc
