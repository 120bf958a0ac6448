#!/bin/bash
# Round-4: x6s with the gfx950 lane-group swizzle (product) against the previous swizzle (libmi3dsparse_prev.so),
# and the conflict-free-read ablation (experiments build, variant 810 vs 10) on the headline rulebooks.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=$GRAFT_REPO_ROOT/3d-weakly-supervised-semantic-segmentation_amd/lib
timeout -k 10 400 python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread tests/test_gpu_ops.py -k "local or tile or wgrad" > gpurun_out/pytest_r04f.log 2>&1 || { tail -30 gpurun_out/pytest_r04f.log; exit 1; }
tail -2 gpurun_out/pytest_r04f.log
for v in prev new prev new; do
  lib=$L/libmi3dsparse.so; [ $v = prev ] && lib=$L/libmi3dsparse_prev.so
  MI3DSPARSE_LIB=$lib LEVELS=1,2,3 PASSES=fwd,bwd FORMS=local N=20 timeout -k 10 300 python -u scripts/kbench.py > gpurun_out/kb_r04f_$v.log 2>&1 || exit 1
  echo "== $v"; grep -E "fwd|bwd" gpurun_out/kb_r04f_$v.log
done
MI3DSPARSE_LIB=$L/libmi3dsparse_exp.so LEVELS=1,2,3 PASSES=fwd,bwd FORMS=x6s_v10,x6s_v810,x6s_v110 EXP_VARIANTS=10,810,110 N=20 timeout -k 10 300 python -u scripts/kbench.py > gpurun_out/kb_r04f_abl.log 2>&1 || exit 1
echo "== ablation"; grep -E "fwd|bwd" gpurun_out/kb_r04f_abl.log
