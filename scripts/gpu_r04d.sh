#!/bin/bash
# Round-4 A/B: the library built with -fno-slp-vectorize (no packed f32 VALU beside the MFMAs) against the
# product build: kernel bench on the headline rulebooks (levels 0-2) for both, then interleaved end-to-end runs.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=$GRAFT_REPO_ROOT/3d-weakly-supervised-semantic-segmentation_amd/lib
LEVELS=0,1,2 FORMS=local,tile,nbr WFORMS=chunk,pairs timeout -k 10 300 python -u scripts/kbench.py > gpurun_out/kb_r04d_A.log 2>&1 || exit 1
MI3DSPARSE_LIB=$L/libmi3dsparse_noslp.so LEVELS=0,1,2 FORMS=local,tile,nbr WFORMS=chunk,pairs timeout -k 10 300 python -u scripts/kbench.py > gpurun_out/kb_r04d_B.log 2>&1 || exit 1
EXP_LIB=$L/libmi3dsparse_noslp.so TAG=r04d_noslp ROUNDS=2 BENCH_ARGS="--steps 15 --warmup 5 --no-cpu" bash scripts/gpu_ab.sh
