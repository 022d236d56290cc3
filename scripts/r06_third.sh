#!/bin/bash
# Round 6, third GPU call: after the CPU staging cache and the launch-order
# fix -- auto vs forced GPU/CPU, parallel readers over 2..4 regions.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -v -s --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_read.py -k "auto_prehash or prehash_rate" > gpurun_out/r06_third_tests.log 2>&1
echo "tests rc=$?"
CASES="rate" OUT_NAME=r06_rate_sweep2 timeout -k 10 500 bash scripts/r06_flush_sweep.sh
