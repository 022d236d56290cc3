#!/bin/bash
# scripts/r04_late_checks.sh -- round 4, late additions on one MI355X: the MD5
# class's copy on a GPU context, the C++ drop-in, the multipart binding
# (cancel flag), then the whole GPU suite once more.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_gpu_parity.py::test_md5_copy_forks_the_state_on_gpu tests/test_gpu_shim.py tests/test_gpu_multipart.py \
  > "$O/r04_late_checks.log" 2>&1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > "$O/r04_gpu_suite_late.log" 2>&1
tail -n 3 "$O/r04_late_checks.log" "$O/r04_gpu_suite_late.log"
