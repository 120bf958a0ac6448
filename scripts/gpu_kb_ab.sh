cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for v in A B; do
  if [ $v = A ]; then export MI3DSPARSE_LIB=$GRAFT_REPO_ROOT/3d-weakly-supervised-semantic-segmentation_amd/lib/libmi3dsparse_exp.so; else unset MI3DSPARSE_LIB; fi
  LEVELS=0,1 PASSES=fwd,bwd,wgrad FORMS=nbr,tile,local N=20 timeout -k 10 400 python -u scripts/kbench.py > gpurun_out/kb0_$v.log 2>&1 || exit $?
  echo "== $v"; tail -12 gpurun_out/kb0_$v.log
done
