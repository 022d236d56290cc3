#!/bin/bash
# scripts/r02_configs_final.sh -- BASELINE configs 1, 3, 4 (+ sweep and split), 5
# (one process and one rank under torch.distributed.run) and the saturation
# lines on the final kernels.  Each step has its own limit; stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u bench_configs.py --configs 1,3,4,4split,5,5h,sat \
  > gpurun_out/configs_final.jsonl 2> gpurun_out/configs_final.err || exit $?
timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
  --master-addr 127.0.0.1 --master-port 29533 bench_config5.py \
  > gpurun_out/config5_n1_final.jsonl 2> gpurun_out/config5_n1_final.err || exit $?
grep -h '^{' gpurun_out/configs_final.jsonl gpurun_out/config5_n1_final.jsonl | cut -c1-260
