#!/bin/bash
# Round-4: local_fill's row grouping with the chosen row's mask broadcast by readlane instead of an LDS read per
# step (lib/libmi3dsparse_exp.so): the tile-local tests and the metadata/prefetch tests on it, then an interleaved
# A/B against the product library.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=$GRAFT_REPO_ROOT/3d-weakly-supervised-semantic-segmentation_amd/lib
MI3DSPARSE_LIB=$L/libmi3dsparse_exp.so timeout -k 10 600 python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_encoders.py -k "local or tile or prefetch or graph or metadata or parity" > gpurun_out/pytest_r04y.log 2>&1 || { tail -30 gpurun_out/pytest_r04y.log; exit 1; }
tail -2 gpurun_out/pytest_r04y.log
TAG=r04y_group ROUNDS=4 BENCH_ARGS="--steps 20 --warmup 5 --no-cpu" bash scripts/gpu_ab.sh || exit 1
