#!/bin/bash
# scripts/r05_gpu_suite.sh -- round 5 on the GPU box: the full -m gpu suite
# (the pull-driven batch, lane-priced routing and load feedback included),
# then the staged multipart sweep (scripts/r05_staged_sweep.sh).  Outputs
# under gpurun_out/r05_*; summaries copied into profiles/.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread \
  > "$O/r05_gpu_suite.log" 2>&1
bash scripts/r05_staged_sweep.sh 2> "$O/r05_staged_sweep.err"
bash scripts/r05_route_sweep.sh > "$O/r05_route_sweep.out" 2> "$O/r05_route_sweep.err"
