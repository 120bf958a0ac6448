set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 LEVELS=5 VARIANTS=2:1:0:0:3,2:1:0:0:2,2:1:0:1:3,2:1:0:1:2
timeout -k 10 300 python scripts/kbench_local.py > gpurun_out/kb_wp_fwd.log 2>&1 && \
FLIP=1 timeout -k 10 300 python scripts/kbench_local.py > gpurun_out/kb_wp_bwd.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/kb_wp_fwd.log gpurun_out/kb_wp_bwd.log; exit $rc
