#!/bin/bash
# scripts/r02_cpu_mb_check.sh -- GPU box check of the multi-buffer CPU backend:
# the -m gpu suite (routing, fallback and sanitizer tests run the CPU backend),
# smoke and bench, then the CPU backend rates on the box's EPYC and config 4
# under auto routing.  Stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
bash scripts/r02_gpu_suite.sh mb || exit $?
timeout -k 10 300 python -u ubench/cpu_mb_rate.py > gpurun_out/cpu_mb_rate.jsonl 2>&1 || exit $?
timeout -k 10 300 python -u bench_configs.py --configs 4split > gpurun_out/mb_4split.jsonl 2>&1 || exit $?
cat gpurun_out/cpu_mb_rate.jsonl; grep '^{' gpurun_out/mb_4split.jsonl | cut -c1-400
