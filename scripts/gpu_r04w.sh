#!/bin/bash
# Round-4: (1) the chunk weight gradient's far rules (msp_wgrad_far_list / msp_conv_wgrad_far) and (2) the
# one-launch small-level BatchNormalization (msp_bn_forward_small / msp_bn_backward_small): their tests, the
# encoder parity and prefetch/graph tests, the per-shape bench, then an interleaved A/B of (2) (B = MSP_BN_SMALL=0).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_encoders.py tests/test_gpu_headline.py -k "wgrad or chunk or prefetch or graph or metadata or parity or batchnorm or bn or join or residual or headline" > gpurun_out/pytest_r04w.log 2>&1 || { tail -30 gpurun_out/pytest_r04w.log; exit 1; }
tail -2 gpurun_out/pytest_r04w.log
MI3DSPARSE_KIND_SHAPES=1 timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu > gpurun_out/bench_r04w_shapes.log 2>&1 || exit 1
TAG=r04w_bnsmall ROUNDS=3 B_LIB=0 BENCH_ARGS="--steps 20 --warmup 5 --no-cpu" B_ENV="MSP_BN_SMALL=0" bash scripts/gpu_ab.sh || exit 1
