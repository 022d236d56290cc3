#!/bin/bash
# scripts/r05_tool.sh -- qsmd5sum over one 5 GiB file (512 parts of 10 MiB),
# mapped (qsmd5_hash_batch) against pulled with pread (--read,
# qsmd5_hash_read), each twice (the second pass finds the file in the page
# cache), then the GPU tool tests.  Output: gpurun_out/r05_tool.log.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
O=gpurun_out/r05_tool.log
F=$(mktemp /tmp/qsmd5sum_XXXX.bin)
python3 -c "
import numpy as np, sys
rng = np.random.default_rng(1)
with open(sys.argv[1], 'wb') as f:
    for _ in range(20):
        f.write(rng.integers(0, 256, size=256 << 20, dtype=np.uint8).tobytes())
" "$F" || exit 1
: > $O
for mode in "" "--read"; do
  for pass in 1 2; do
    t0=$(date +%s%N)
    timeout -k 10 120 qsfs-fuse_amd/bin/qsmd5sum $mode --parts "$F" > /tmp/qsmd5sum_out_$pass.txt || exit 1
    t1=$(date +%s%N)
    echo "mode=${mode:-mapped} pass=$pass seconds=$(( (t1 - t0) / 1000000 ))e-3 parts=$(wc -l < /tmp/qsmd5sum_out_$pass.txt) digest_of_output=$(md5sum < /tmp/qsmd5sum_out_$pass.txt | cut -c1-32)" >> $O
  done
done
rm -f "$F"
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_tools.py >> $O 2>&1
