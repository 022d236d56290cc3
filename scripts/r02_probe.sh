#!/bin/bash
# Round-2 probes (run through gpurun): sanitizer tests; pageable-pool staging
# through the multipart harness under /opt/rocm's HIP and under torch's HIP;
# config 3 from pageable memory in Python; config 5 at N = 1 (bench_config5.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02g
mkdir -p $O
TL=$(python -c "import torch,os;print(os.path.dirname(torch.__file__)+'/lib')")
timeout -k 10 300 python -u -m pytest tests/test_gpu_sanitizers.py -m gpu -v --timeout 200 \
  --timeout-method thread > $O/san.log 2>&1 || { tail -5 $O/san.log; exit 1; }
tail -2 $O/san.log
H="tests/cpp/multipart_harness --aligned --size=$((512*10485760)) --pool=512"
for slab in "" "--slab"; do
  QSMD5_BACKEND=gpu QSMD5_TRACE=1 timeout -k 10 120 $H $slab > $O/h_rocm${slab}.json 2> $O/h_rocm${slab}.trace || exit 1
  QSMD5_BACKEND=gpu QSMD5_TRACE=1 LD_LIBRARY_PATH=$TL timeout -k 10 120 $H $slab > $O/h_torch${slab}.json 2> $O/h_torch${slab}.trace || exit 1
done
for f in $O/h_*.json; do echo "$f $(python -c "import json,sys;d=json.load(open('$f'));print('hash_s',d['hash_s'],'GiB/s',round(5/d['hash_s'],1))")"; done
timeout -k 10 200 python -u bench_configs.py --configs 3p --reps 2 > $O/cfg3p.jsonl 2> $O/cfg3p.err || exit 1
cat $O/cfg3p.jsonl
timeout -k 10 400 python -u bench_config5.py --reps 2 > $O/cfg5.jsonl 2> $O/cfg5.err || { tail $O/cfg5.err; exit 1; }
cat $O/cfg5.jsonl
for nt in 0 1; do
  QSMD5_LOAD_NT=$nt QSMD5_SWEEP_EXTRA_MIB=24,48,96,128 timeout -k 10 400 python -u bench_configs.py --configs 4 --reps 2 \
    > $O/sweep_nt$nt.jsonl 2> $O/sweep_nt$nt.err || { tail $O/sweep_nt$nt.err; exit 1; }
  tail -1 $O/sweep_nt$nt.jsonl
done
