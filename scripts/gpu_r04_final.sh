#!/bin/bash
# Round-4 closing session: smoke, the GPU suite, the default bench line, the rocprofv3 kernel trace + stats of the
# bench (profiles/r04/kernel_stats_*), the PMC traffic of the conv family (profiles/r04/pmc_traffic.json) and the
# per-kernel PMC summary.  Each GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-r04final}
STEPS=${STEPS:-smoke,test,bench,prof,traffic,pmc}
for st in ${STEPS//,/ }; do
  case $st in
    smoke) timeout -k 10 300 python -c "import __graft_entry__ as g; g.add_path(); g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1; rc=$?; tail -2 gpurun_out/smoke_$TAG.log ;;
    test) timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -s --timeout 900 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu_$TAG.log ;;
    bench) timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_$TAG.log 2>&1; rc=$?; tail -1 gpurun_out/bench_$TAG.log | cut -c1-600 ;;
    prof) TAG=$TAG bash scripts/gpu_profile_r03.sh > gpurun_out/profsum_$TAG.log 2>&1; rc=$?; head -40 gpurun_out/profsum_$TAG.log ;;
    traffic) TAG=$TAG bash scripts/pmc_traffic.sh > gpurun_out/traffic_$TAG.log 2>&1; rc=$?; tail -5 gpurun_out/traffic_$TAG.log ;;
    pmc) TAG=pmc$TAG bash scripts/gpu_pmc_r03.sh > gpurun_out/pmcrun_$TAG.log 2>&1; rc=$?; tail -5 gpurun_out/pmcrun_$TAG.log ;;
    *) echo "unknown step $st"; rc=2 ;;
  esac
  echo "== step $st rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
