#!/bin/bash
# scripts/r02_lanes_check.sh -- GPU box: the -m gpu suite, smoke and bench on
# the final tree, then BASELINE config 4 under auto routing with the lanes
# priced (QSMD5_ROUTE_LANES=1) and the CPU backend rates.  Stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
bash scripts/r02_gpu_suite.sh lanes || exit $?
QSMD5_ROUTE_LANES=1 timeout -k 10 300 python -u bench_configs.py --configs 4split \
  > gpurun_out/lanes_4split.jsonl 2>&1 || exit $?
grep '^{' gpurun_out/lanes_4split.jsonl | cut -c1-400
