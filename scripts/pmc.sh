#!/bin/bash
# PMC counter passes (one rocprofv3 run per pass, kernel-trace only beside
# --pmc) over a command.  Output: gpurun_out/pmc_<tag>/pass<i>/.
#   TAG=r01 PASSES="FETCH_SIZE|WRITE_SIZE" ./scripts/pmc.sh python3 bench.py --steps 2 --warmup 1 --no-cpu
set -o pipefail
TAG=${TAG:-r01}
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc_${TAG}
IFS='|' read -ra P <<< "${PASSES:-FETCH_SIZE|WRITE_SIZE}"
i=0
for pass in "${P[@]}"; do
  timeout -k 10 ${PASS_TIMEOUT:-300} rocprofv3 --pmc ${pass} --kernel-trace --output-format csv \
    -d gpurun_out/pmc_${TAG}/pass${i} -o run -- "$@" > gpurun_out/pmc_${TAG}/pass${i}.log 2>&1 || exit $?
  echo "pass $i ($pass) ok"
  i=$((i + 1))
done
