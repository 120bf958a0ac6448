# Pair-list weight gradient: timing ablations (msp_debug_wgrad_abl bits: 1 no splits, 2 no MFMAs,
# 4 no row loads, 8 no pair-list loads), more pieces, and PMC passes over the default form.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 MODES=0
for abl in ${ABLS:-0 1 2 4 8 12 15}; do
  echo "== ABL=$abl"
  ABL=$abl timeout -k 10 180 python scripts/kbench_wgrad.py 2>&1 | grep -v amdgpu.ids || exit 1
done
echo "== BLOCKS=16384"
BLOCKS=16384 timeout -k 10 180 python scripts/kbench_wgrad.py 2>&1 | grep -v amdgpu.ids || exit 1
if [ -n "$PMC" ]; then
  TAG=wgrad PASSES="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE|TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum GRBM_GUI_ACTIVE|FETCH_SIZE GRBM_GUI_ACTIVE|TA_BUSY_avr TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum GRBM_GUI_ACTIVE" \
    PASS_TIMEOUT=180 bash scripts/pmc.sh python3 scripts/kbench_wgrad.py && \
    python3 scripts/pmc_dispatch.py gpurun_out/pmc_wgrad wgrad_x6_kernel > gpurun_out/pmc_wgrad.txt && cat gpurun_out/pmc_wgrad.txt
fi
