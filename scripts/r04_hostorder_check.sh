#!/bin/bash
# scripts/r04_hostorder_check.sh -- round 4: the host-ordered staging pipeline
# (no hipStreamWaitEvent between copy and compute streams) on the GPU box:
# the staging / column / multipart / parity / config-5 tests, host-resident
# config 3 (4096 x 10 MiB pinned) and 3cmp throughput, and the spinning-thread
# probe of the multipart harness.  Outputs under gpurun_out/r04_hostorder_*.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_staging.py tests/test_gpu_columns.py tests/test_gpu_multipart.py tests/test_gpu_parity.py \
  tests/test_gpu_fuzz.py tests/test_gpu_multi.py tests/test_gpu_routing.py tests/test_gpu_coalesce.py \
  > "$O/r04_hostorder_tests.log" 2>&1
timeout -k 10 600 python -u bench_configs.py --configs 3,3cmp,4 > "$O/r04_hostorder_configs.jsonl" 2> "$O/r04_hostorder_configs.err"
bash scripts/r04_spin_thread_probe.sh > /dev/null
cp "$O/r04_spin_thread_probe.log" "$O/r04_hostorder_spin.log"
tail -3 "$O/r04_hostorder_tests.log"
cat "$O/r04_hostorder_configs.jsonl" "$O/r04_hostorder_spin.log"
