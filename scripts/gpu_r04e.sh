#!/bin/bash
# Round-4 A/B: level 0's 32 x 32 weight gradients on the chunk-local form over a lists-only tile-local rulebook
# (A, product) against the pair lists (B: the same sources with -DMSP_CHUNK_NARROW=0); GPU tests of the touched
# paths first.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -m gpu -x -v -s --timeout 500 --timeout-method thread tests/test_gpu_fullsize.py tests/test_gpu_encoders.py tests/test_gpu_weight_images.py > gpurun_out/pytest_r04e.log 2>&1 || { tail -30 gpurun_out/pytest_r04e.log; exit 1; }
tail -3 gpurun_out/pytest_r04e.log
TAG=r04e_l0chunk ROUNDS=3 BENCH_ARGS="--steps 15 --warmup 5 --no-cpu" bash scripts/gpu_ab.sh
