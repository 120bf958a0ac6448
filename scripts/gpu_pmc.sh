#!/bin/bash
# PMC passes over the eager bench (2 timed steps): MFMA busy, wait states, LDS activity and bank
# conflicts, instruction mix, L2 hits per dispatch of the conv / wgrad / BN kernels.
# Usage (GPU box): TAG=x bash scripts/gpu_pmc.sh
set -o pipefail
TAG=${TAG:-r03a}
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
P0="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
P1="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVES SQ_WAIT_INST_LDS SQ_BUSY_CYCLES TCC_HIT_sum TCC_MISS_sum"
PASSES="$P0|$P1" TAG=$TAG PASS_TIMEOUT=240 bash scripts/pmc.sh python3 bench.py --steps 2 --warmup 1 --no-cpu --graph 0 --record none --family-steps 1 || exit $?
for f in conv_x6s conv_x6r conv_x6g conv_x6d wgrad_x6_kernel wgrad_x6c bn_ nin_gemm conv_pairs; do
  echo "== $f"; python3 scripts/pmc_dispatch.py gpurun_out/pmc_$TAG "$f"
done > gpurun_out/pmc_${TAG}_summary.txt
cat gpurun_out/pmc_${TAG}_summary.txt | cut -c1-400
