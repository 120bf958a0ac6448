#!/bin/bash
# PMC HBM traffic of msp_conv_tile on the bench workload: FETCH_SIZE and
# WRITE_SIZE in two separate rocprofv3 runs (kernel trace only beside --pmc),
# summarised to gpurun_out/pmc_traffic_<tag>.json.
set -o pipefail
TAG=${TAG:-r01}
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
PASSES="FETCH_SIZE|WRITE_SIZE" TAG=traffic_${TAG} PASS_TIMEOUT=${PASS_TIMEOUT:-300} \
  bash scripts/pmc.sh python3 bench.py --steps 2 --warmup 1 --no-cpu && \
  python3 scripts/pmc_traffic.py gpurun_out/pmc_traffic_${TAG} gpurun_out/pmc_traffic_${TAG}.json
