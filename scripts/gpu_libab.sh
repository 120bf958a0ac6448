#!/bin/bash
# Parity of the experiment build (lib/libmi3dsparse_exp.so, scripts/build_exp.sh with EXP_FLAGS) against the
# product build on the full-size and conv-accuracy GPU tests (errors printed), then an interleaved bench A/B.
# TAG names the outputs under gpurun_out/; PYTEST_K selects tests; ROUNDS bench rounds (0: no bench).
set -o pipefail
TAG=${TAG:-libab}
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
EXP=$GRAFT_REPO_ROOT/3d-weakly-supervised-semantic-segmentation_amd/lib/libmi3dsparse_exp.so
for v in A B; do
  if [ $v = B ]; then export MI3DSPARSE_LIB=$EXP; else unset MI3DSPARSE_LIB; fi
  timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_ops.py -m gpu -x -v -s \
    --timeout 300 --timeout-method thread -k "${PYTEST_K:-fullsize or accuracy or subm_conv}" \
    > gpurun_out/libab_${TAG}_$v.log 2>&1; rc=$?
  echo "== $v pytest rc=$rc"; grep -E "max err|worst|passed|failed" gpurun_out/libab_${TAG}_$v.log | tail -12
  [ $rc -eq 0 ] || exit $rc
done
unset MI3DSPARSE_LIB
if [ "${ROUNDS:-2}" != 0 ]; then TAG=$TAG ROUNDS=${ROUNDS:-2} bash scripts/gpu_ab.sh; fi
