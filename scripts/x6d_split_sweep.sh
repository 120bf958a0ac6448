#!/bin/bash
# conv_x6d's split-K plan on the small levels (the shared-tile form, levels 4-6): kbench's "tile" form on the
# experiment build for several (target blocks, cap) settings, MSP_X6D_SPLIT="target_small,cap_small,target,cap"
# (n_tiles <= 8 takes the first pair).  One log per setting under gpurun_out/x6d_split_$TAG/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-sweep}
mkdir -p gpurun_out/x6d_split_$TAG
export MI3DSPARSE_LIB=$GRAFT_REPO_ROOT/3d-weakly-supervised-semantic-segmentation_amd/lib/libmi3dsparse_exp.so
for cfg in ${CFGS:-2048,16,1024,8 1024,8,512,4 4096,32,2048,16 512,4,256,2 1,1,1,1}; do
  MSP_X6D_SPLIT=$cfg LEVELS=${LEVELS:-4,5,6} PASSES=fwd,bwd FORMS=tile N=${N:-30} timeout -k 10 200 \
    python -u scripts/kbench.py > gpurun_out/x6d_split_$TAG/$cfg.log 2>&1 || exit $?
  echo "== $cfg"; grep -E "^L|tile" gpurun_out/x6d_split_$TAG/$cfg.log
done
