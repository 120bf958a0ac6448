# Chunk-local conv micro-benchmark (fwd and bwd-data layouts).
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 240 python scripts/kbench_chunk.py > gpurun_out/kbench_chunk.log 2>&1 \
  && FLIP=1 timeout -k 10 240 python scripts/kbench_chunk.py > gpurun_out/kbench_chunk_bwd.log 2>&1
rc=$?
grep -v amdgpu.ids gpurun_out/kbench_chunk.log; grep -v amdgpu.ids gpurun_out/kbench_chunk_bwd.log 2>/dev/null
exit $rc
