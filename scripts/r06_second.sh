#!/bin/bash
# Round 6, second GPU call: routing with clean/busy read rates and the
# pre-allocated read slot (auto vs forced GPU), parallel readers over 2..4
# staging regions, the nested-callback tests.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -v -s --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_read.py -k "auto_prehash or call_back or prehash_rate or staged_prehash_default" \
  > gpurun_out/r06_second_tests.log 2>&1
echo "tests rc=$?"
CASES="auto rate" OUT_NAME=r06_rate_sweep timeout -k 10 500 bash scripts/r06_flush_sweep.sh
