#!/bin/bash
# scripts/r04_gpu_suite.sh -- round 4 on the GPU box: the full -m gpu suite,
# smoke(), and the default bench line (run through gpurun; outputs under
# gpurun_out/, summaries copied into profiles/r04_*).
set -euo pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread \
  > "$O/r04_gpu_suite.log" 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/r04_smoke.log" 2>&1
timeout -k 10 600 python -u bench.py > "$O/r04_bench.json" 2> "$O/r04_bench.err"
