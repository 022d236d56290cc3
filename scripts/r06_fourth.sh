#!/bin/bash
# Round 6, fourth GPU call: the flush sweep on the tree with read-ahead,
# adaptive background waves, clean/busy routing and the CPU staging cache;
# the ramp and reference-loop tests.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -v -s --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_read.py tests/test_gpu_multipart.py -k "ramp or reference_loop" > gpurun_out/r06_fourth_tests.log 2>&1
echo "tests rc=$?"
OUT_NAME=r06_flush_sweep_final timeout -k 10 900 bash scripts/r06_flush_sweep.sh
