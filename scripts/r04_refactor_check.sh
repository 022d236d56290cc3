#!/bin/bash
# scripts/r04_refactor_check.sh -- round 4, after splitting the host runtime into
# units (qsmd5_rt.h): the whole GPU suite, smoke(), and the default bench line.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > "$O/r04_gpu_suite_split.log" 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/r04_smoke_split.log" 2>&1
timeout -k 10 600 python -u bench.py > "$O/r04_bench_split.json" 2> "$O/r04_bench_split.err"
tail -n 2 "$O/r04_gpu_suite_split.log"
python3 -c "import json; r=json.load(open('$O/r04_bench_split.json')); print(r['value'], r['ms_per_step'], r['config5_host']['value'], r['parity'])"
