#!/bin/bash
# Experiment build: lib/libmi3dsparse_exp.so = the product sources compiled with -DMSP_EXPERIMENTS (adds the
# msp_exp_* kernel-variant entries scripts/kbench.py measures).  The product library is built without them.
set -e
cd "$(dirname "$0")/../3d-weakly-supervised-semantic-segmentation_amd/csrc"
mkdir -p ../build/exp
OBJS=""
PIDS=""
for f in msp_core msp_meta msp_conv msp_bn msp_layers msp_tail msp_merge msp_conv_x6 msp_nin msp_local msp_sort msp_optim; do
  extra=""
  case $f in msp_conv_x6|msp_local) extra="-mllvm -amdgpu-mfma-vgpr-form" ;; esac
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -Wall -Wno-unused-function -I/opt/rocm/include \
    -DMSP_EXPERIMENTS ${EXP_FLAGS:-} $extra -c $f.hip -o ../build/exp/$f.o &
  PIDS="$PIDS $!"
  OBJS="$OBJS ../build/exp/$f.o"
done
for p in $PIDS; do wait $p; done  # a failed compile fails the build (set -e)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $OBJS -o ../lib/libmi3dsparse_exp.so
echo built ../lib/libmi3dsparse_exp.so
