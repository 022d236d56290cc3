#!/bin/bash
# Round 5, first GPU call: the new self-launch / digest-isolation tests, the
# oracle-anchored shim/tools/etag tests, then the default bench line.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_process.py tests/test_gpu_shim.py tests/test_gpu_tools.py \
  "tests/test_gpu_parity.py::test_verify_etag_download_buffer" \
  > gpurun_out/r05_first_tests.log 2>&1 &&
timeout -k 10 600 python -u bench.py > gpurun_out/r05_bench_first.json 2> gpurun_out/r05_bench_first.err
