#!/bin/bash
# PMC passes over the conv_tile micro-benchmark (scripts/kbench_conv.py);
# one rocprofv3 run per pass.  Output: gpurun_out/pmc_<tag>/pass<i>/ and a
# per-dispatch summary in gpurun_out/pmc_<tag>.txt.
set -o pipefail
TAG=${TAG:-kb}
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
export PASSES=${PASSES:-"SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE|TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum GRBM_GUI_ACTIVE|FETCH_SIZE GRBM_GUI_ACTIVE|WRITE_SIZE TA_BUSY_avr TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum GRBM_GUI_ACTIVE"}
TAG=$TAG PASS_TIMEOUT=${PASS_TIMEOUT:-240} bash scripts/pmc.sh python3 "$@" && \
  python3 scripts/pmc_dispatch.py gpurun_out/pmc_${TAG} ${FILTER:-conv_tile} > gpurun_out/pmc_${TAG}.txt
