#!/bin/bash
# Round 5: the pull-driven batch on the GPU (tests/test_gpu_read.py), then the
# staged multipart sweep (scripts/r05_staged_sweep.sh).
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_read.py \
  > gpurun_out/r05_gpu_read_tests.log 2>&1 &&
bash scripts/r05_staged_sweep.sh 2> gpurun_out/r05_staged_sweep.err
