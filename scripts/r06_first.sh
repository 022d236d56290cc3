#!/bin/bash
# Round 6, first GPU call: the new read-path tests (nested callbacks, auto vs
# forced GPU, parallel-reader rates, reference loop beside the binding), then
# the flush sweep (scripts/r06_flush_sweep.sh).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -v -s --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_read.py tests/test_gpu_multipart.py > gpurun_out/r06_first_tests.log 2>&1
echo "tests rc=$?"
timeout -k 10 500 bash scripts/r06_flush_sweep.sh
