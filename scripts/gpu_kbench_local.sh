# Tile-local conv micro-benchmark (fwd and bwd-data layouts) + one SQ PMC pass over it.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python scripts/kbench_local.py > gpurun_out/kbench_local.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/kbench_local.log
[ $rc -eq 0 ] || exit $rc
if [ -n "$PMC" ]; then export VARIANTS=${PMC_VARIANTS:-2:1:0}
  TAG=local PASSES="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE" \
    LEVELS=3 bash scripts/pmc.sh python3 scripts/kbench_local.py && \
    python3 scripts/pmc_dispatch.py gpurun_out/pmc_local conv_x6s > gpurun_out/pmc_local.txt && cat gpurun_out/pmc_local.txt
fi
