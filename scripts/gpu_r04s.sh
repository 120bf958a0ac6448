#!/bin/bash
# Round-4: graph-replay gap probe (is the ~1 ms before each step's replay the graph launch itself?).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/graph_gap_probe.py > gpurun_out/graph_gap_probe_r04s.log 2>&1 || { cat gpurun_out/graph_gap_probe_r04s.log; exit 1; }
cat gpurun_out/graph_gap_probe_r04s.log
