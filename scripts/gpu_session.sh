#!/bin/bash
# The one GPU-session runner (replaces the per-session scripts/gpu_r0*.sh of rounds 1-4).  Runs the comma-separated
# STEPS in order on the gpurun box, each under its own time limit, and stops at the first failing step.  Outputs go
# to gpurun_out/<step>_$TAG.log (TAG names the session).
#
#   smoke    __graft_entry__.smoke()
#   test     the GPU suite (PYTEST_K selects tests, PYTEST_FILES the files; default: all of tests/ -m gpu)
#   bench    bench.py (BENCH_ARGS, default --gpus 1 --steps 20 --warmup 5)
#   prof     rocprofv3 kernel trace + stats of the bench (scripts/gpu_profile.sh)
#   traffic  PMC FETCH_SIZE / WRITE_SIZE of the conv family (scripts/pmc_traffic.sh)
#   pmc      per-kernel PMC summary (scripts/gpu_pmc.sh)
#   kbench   scripts/kbench.py on the product library (LEVELS / PASSES / FORMS / X6R_VARIANTS ... passed through)
#   kbexp    scripts/kbench.py on the experiments build (lib/libmi3dsparse_exp.so, scripts/build_exp.sh)
#   ab       interleaved end-to-end A/B of the product and experiments builds (scripts/gpu_ab.sh)
#   args     interleaved bench.py argument sets ARGS_0.. (scripts/gpu_args_ab.sh)
#   n2gloo   the two-rank shared-device rehearsal of bench.py's N>1 path with per-rank host timing
#   presets  bench.py --preset c2 / c4 / c5
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-s}
STEPS=${STEPS:-smoke,test,bench}
EXP=$GRAFT_REPO_ROOT/3d-weakly-supervised-semantic-segmentation_amd/lib/libmi3dsparse_exp.so
for st in ${STEPS//,/ }; do
  log=gpurun_out/${st}_$TAG.log
  case $st in
    smoke) timeout -k 10 300 python -c "import __graft_entry__ as g; g.add_path(); g.smoke()" > $log 2>&1; rc=$?
           tail -2 $log ;;
    test) timeout -k 10 1100 python -u -m pytest ${PYTEST_FILES:-tests} -m gpu -x -v -s --timeout 900 \
            --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $log 2>&1; rc=$?
          tail -3 $log ;;
    bench) timeout -k 10 400 python -u bench.py ${BENCH_ARGS:---gpus 1 --steps 20 --warmup 5} > $log 2>&1; rc=$?
           tail -1 $log | cut -c1-700 ;;
    prof) TAG=$TAG bash scripts/gpu_profile.sh > $log 2>&1; rc=$?; head -45 $log ;;
    traffic) TAG=$TAG bash scripts/pmc_traffic.sh > $log 2>&1; rc=$?; tail -5 $log ;;
    pmc) TAG=pmc$TAG bash scripts/gpu_pmc.sh > $log 2>&1; rc=$?; tail -5 $log ;;
    kbench) unset MI3DSPARSE_LIB; timeout -k 10 500 python -u scripts/kbench.py > $log 2>&1; rc=$?; tail -40 $log ;;
    kbexp) MI3DSPARSE_LIB=$EXP timeout -k 10 500 python -u scripts/kbench.py > $log 2>&1; rc=$?; tail -40 $log ;;
    ab) TAG=$TAG bash scripts/gpu_ab.sh > $log 2>&1; rc=$?; cat $log ;;
    args) TAG=$TAG bash scripts/gpu_args_ab.sh > $log 2>&1; rc=$?; cat $log ;;
    n2gloo) BENCH_BACKEND=gloo BENCH_SHARE_DEVICE=1 BENCH_HOST_TIMING=1 timeout -k 10 600 \
              python -u bench.py --gpus 2 ${N2_ARGS:---steps 6 --warmup 2} > $log 2>&1; rc=$?
            tail -30 $log | cut -c1-900 ;;
    presets) rc=0
             for p in c2 c4 c5; do
               timeout -k 10 400 python -u bench.py --preset $p --steps 15 --warmup 5 > gpurun_out/preset_${p}_$TAG.log 2>&1 \
                 || { rc=$?; break; }
               tail -1 gpurun_out/preset_${p}_$TAG.log | cut -c1-300
             done ;;
    *) echo "unknown step $st"; rc=2 ;;
  esac
  echo "== step $st rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
