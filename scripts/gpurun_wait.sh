#!/bin/bash
# Local helper (runs here, not on the box): re-issue a gpurun call only while the pod has no free GPU slot
# (gpurun exit 3 / "all GPU slots busy": nothing ran, nothing charged).  Any other outcome is final.
# Usage: scripts/gpurun_wait.sh <log> <gpurun args...>
# retry gpurun only while no slot/box is free (exit 3); any other outcome is final
out=$1; shift
for i in $(seq 1 40); do
  /usr/local/graft/bin/gpurun "$@" > "$out" 2>&1
  rc=$?
  if [ $rc -ne 3 ] && ! grep -q "all 4 GPU slot" "$out"; then exit $rc; fi
  sleep 90
done
exit 3
