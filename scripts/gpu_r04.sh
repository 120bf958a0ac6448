#!/bin/bash
# Round-4 GPU session: STEPS (comma list) of test | kbench | pmc | bench | prof, each under its own time limit,
# stopping at the first failure.  Outputs under gpurun_out/ (TAG names them).
set -o pipefail
TAG=${TAG:-r04}
STEPS=${STEPS:-test,kbench,pmc}
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for st in ${STEPS//,/ }; do
  case $st in
    test)
      timeout -k 10 1500 python -u -m pytest -m gpu -x -v -s --timeout 1200 --timeout-method thread ${PYTEST_FILES:-tests} ${PYTEST_K:+-k "$PYTEST_K"} \
        > gpurun_out/pytest_gpu_$TAG.log 2>&1; rc=$?; tail -5 gpurun_out/pytest_gpu_$TAG.log ;;
    kbench)
      timeout -k 10 400 python -u scripts/kbench.py > gpurun_out/kbench_$TAG.log 2>&1; rc=$?; cat gpurun_out/kbench_$TAG.log | tail -40 ;;
    kbexp)  # the experiment build's kernel variants (lib/libmi3dsparse_exp.so, scripts/build_exp.sh)
      MI3DSPARSE_LIB=$GRAFT_REPO_ROOT/3d-weakly-supervised-semantic-segmentation_amd/lib/libmi3dsparse_exp.so \
        timeout -k 10 400 python -u scripts/kbench.py > gpurun_out/kbexp_$TAG.log 2>&1; rc=$?; cat gpurun_out/kbexp_$TAG.log | tail -40 ;;
    pmc)
      TAG=$TAG bash scripts/gpu_pmc_r03.sh; rc=$? ;;
    bench)
      timeout -k 10 400 python -u bench.py ${BENCH_ARGS:-} > gpurun_out/bench_$TAG.log 2>&1; rc=$?; tail -3 gpurun_out/bench_$TAG.log | cut -c1-3000 ;;
    prof)
      TAG=$TAG bash scripts/gpu_profile_r03.sh > gpurun_out/profsum_$TAG.log 2>&1; rc=$?; tail -40 gpurun_out/profsum_$TAG.log ;;
    *) echo "unknown step $st"; rc=2 ;;
  esac
  echo "== step $st rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
