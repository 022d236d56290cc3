#!/bin/bash
# scripts/r02_lead_check.sh -- GPU check of the graded phase-start wait (kPcLead):
# the -m gpu suite, smoke, bench, and the ubench A/B (lead vs none, and the
# kernel-selection sweep that runs the 64 KiB-ring kernel).  Stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
bash scripts/r02_gpu_suite.sh lead || exit $?
timeout -k 10 300 ./ubench/ubench_md5 lead > gpurun_out/lead_ab.log 2>&1 || exit $?
timeout -k 10 300 ./ubench/ubench_md5 cross > gpurun_out/lead_cross.log 2>&1 || exit $?
tail -12 gpurun_out/lead_ab.log
