#!/bin/bash
# Round-4 experiment: s_setprio 2 around conv_x6s's per-group MFMAs (lib/libmi3dsparse_exp.so built with
# -DMSP_X6S_SETPRIO=1) against the product: kbench of the tile-local form, both orders, then end to end.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=$GRAFT_REPO_ROOT/3d-weakly-supervised-semantic-segmentation_amd/lib
for v in A B B2 A2; do
  lib=""; case $v in B*) lib="MI3DSPARSE_LIB=$L/libmi3dsparse_exp.so";; esac
  env $lib LEVELS=1,2,3 PASSES=fwd,bwd FORMS=local N=20 timeout -k 10 300 python -u scripts/kbench.py > gpurun_out/kb_r04ab_$v.log 2>&1 || exit 1
done
grep -h "local" gpurun_out/kb_r04ab_A.log gpurun_out/kb_r04ab_B.log gpurun_out/kb_r04ab_B2.log gpurun_out/kb_r04ab_A2.log
TAG=r04ab_setprio ROUNDS=2 BENCH_ARGS="--steps 20 --warmup 5 --no-cpu" bash scripts/gpu_ab.sh || exit 1
