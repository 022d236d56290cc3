#!/bin/bash
# scripts/r04_final.sh -- round 4's evidence on one MI355X: the full -m gpu
# suite, smoke(), the default bench line, then scripts/profile_round.sh's
# rocprofv3 passes (kernel trace + stats of bench.py, FETCH_SIZE passes, the
# saturation lines).  Summaries: python3 scripts/summarize_profiles.py r04.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > "$O/r04_gpu_suite_final.log" 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/r04_smoke_final.log" 2>&1
timeout -k 10 600 python -u bench.py > "$O/r04_bench_final.json" 2> "$O/r04_bench_final.err"
bash scripts/profile_round.sh
tail -3 "$O/r04_gpu_suite_final.log"
