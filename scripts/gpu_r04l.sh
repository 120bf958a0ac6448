#!/bin/bash
# Round-4: conv_x6sc (column halves: every weight fragment serves all 8 row groups, next step's fragments in
# flight during the step) against conv_x6s, on the headline batch's rulebooks.  A = product library (x6s, per-half
# lists); B = experiments build with -DMSP_SHARED_LISTS=1: x6s over shared lists ("local"), x6sc (v2000), x6sc
# over round-robin offsets (v2001), x6sc without weight loads past the first step (v2400, ablation).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=$GRAFT_REPO_ROOT/3d-weakly-supervised-semantic-segmentation_amd/lib
for i in 1 2; do
  LEVELS=1,2,3,4 PASSES=fwd,bwd FORMS=local N=20 timeout -k 10 300 python -u scripts/kbench.py > gpurun_out/kb_r04l_A$i.log 2>&1 || exit 1
  MI3DSPARSE_LIB=$L/libmi3dsparse_exp.so LEVELS=1,2,3,4 PASSES=fwd,bwd FORMS=local,x6s_v2000,x6s_v2001,x6s_v2400 EXP_VARIANTS=2000,2001,2400 N=20 timeout -k 10 300 python -u scripts/kbench.py > gpurun_out/kb_r04l_B$i.log 2>&1 || exit 1
done
cat gpurun_out/kb_r04l_A1.log gpurun_out/kb_r04l_B1.log
