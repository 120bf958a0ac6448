#!/bin/bash
# Round-4 experiment: the chunk weight gradient with 2x / 3x more (shorter) tile ranges than one block per CU
# (MSP_WGRAD_RANGES_MULT): interleaved A/Bs against the product.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=r04aa_ranges2 ROUNDS=3 B_LIB=0 BENCH_ARGS="--steps 20 --warmup 5 --no-cpu" B_ENV="MSP_WGRAD_RANGES_MULT=2" bash scripts/gpu_ab.sh || exit 1
TAG=r04aa_ranges3 ROUNDS=2 B_LIB=0 BENCH_ARGS="--steps 20 --warmup 5 --no-cpu" B_ENV="MSP_WGRAD_RANGES_MULT=3" bash scripts/gpu_ab.sh || exit 1
