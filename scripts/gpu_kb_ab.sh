#!/bin/bash
# kbench.py on the experiment build (A: lib/libmi3dsparse_exp.so) and on the product build (B), one after the
# other on one box.  LEVELS / PASSES / FORMS as kbench.py; outputs gpurun_out/kb_${TAG}_{A,B}.log.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
TAG=${TAG:-kb}
for v in A B; do
  if [ $v = A ]; then export MI3DSPARSE_LIB=$GRAFT_REPO_ROOT/3d-weakly-supervised-semantic-segmentation_amd/lib/libmi3dsparse_exp.so; else unset MI3DSPARSE_LIB; fi
  LEVELS=${LEVELS:-0,1} PASSES=${PASSES:-fwd,bwd,wgrad} FORMS=${FORMS:-nbr,tile,local} N=${N:-20} \
    timeout -k 10 400 python -u scripts/kbench.py > gpurun_out/kb_${TAG}_$v.log 2>&1 || exit $?
  echo "== $v"; tail -14 gpurun_out/kb_${TAG}_$v.log
done
