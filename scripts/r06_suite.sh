#!/bin/bash
# scripts/r06_suite.sh TAG -- round 6 on one MI355X: the full -m gpu suite,
# smoke(), and the default bench line; outputs gpurun_out/r06_{gpu_suite,smoke,bench}_TAG.*
set -uo pipefail
T=${1:-final}
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread \
  > "$O/r06_gpu_suite_$T.log" 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/r06_smoke_$T.log" 2>&1 || exit 1
timeout -k 10 600 python -u bench.py > "$O/r06_bench_$T.json" 2> "$O/r06_bench_$T.err"
