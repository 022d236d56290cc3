#!/bin/bash
# Round 5: the pool-free pre-hash (qsmd5::upload_parts_staged over qsmd5_hash_read)
# against round 4's pool-bound waves, inside DoMultiPartUpload at qsfs's default
# -n 5 and beyond.  A file of P x 10 MiB parts held in pages
# (part i = LCG(12345 + i), every digest checked against the golden table by the
# caller), QSMD5_BACKEND=auto, second pass reported (--repeat=2).
# Output: gpurun_out/r05_staged_sweep.jsonl, one harness JSON per line with a
# "case" key.
set -o pipefail
mkdir -p gpurun_out
OUT=gpurun_out/r05_staged_sweep.jsonl
: > $OUT
H=tests/cpp/multipart_harness
run() {  # case-name, args...
  local name=$1; shift
  timeout -k 10 300 env QSMD5_BACKEND=${BACKEND:-auto} $H --aligned --repeat=2 "$@" > gpurun_out/_one.json || return 1
  python3 - "$name" >> $OUT <<'PY'
import json, sys
r = json.load(open("gpurun_out/_one.json"))
gold = json.load(open("tests/golden/batch_10MiB.json"))["md5"]
r["case"] = sys.argv[1]
r["golden_ok"] = all(m == gold[:len(m)] for m in r["md5_files"])
for k in ("md5", "md5_files", "part_sizes"):
    r.pop(k, None)
print(json.dumps(r))
PY
  echo "$name done" >&2
}
for P in 128 512; do
  S=$((P * 10 * 1024 * 1024))
  run "waves_n5_P$P" --size=$S --pool=5 --pinned --no-pipeline || exit 1
  run "staged_n5_P$P" --size=$S --pool=5 --pinned --staged || exit 1
  BACKEND=gpu run "staged_n5_gpu_P$P" --size=$S --pool=5 --pinned --staged || exit 1
  BACKEND=cpu run "staged_n5_cpu_P$P" --size=$S --pool=5 --pinned --staged || exit 1
  run "staged_n5_pageable_pool_P$P" --size=$S --pool=5 --staged || exit 1
  for B in 64 1024; do
    run "staged_n5_staging${B}M_P$P" --size=$S --pool=5 --pinned --staged --staging=$((B << 20)) || exit 1
  done
  run "staged_n5_waves64_P$P" --size=$S --pool=5 --pinned --staged --wave-parts=64 || exit 1
  run "staged_n5_upload10ms_P$P" --size=$S --pool=5 --pinned --staged --wave-parts=64 --upload-ms=10 || exit 1
  run "staged_n5_ramp4_upload10ms_P$P" --size=$S --pool=5 --pinned --staged --wave-parts=64 --first-wave=4 --upload-ms=10 || exit 1
  run "staged_n5_ramp4_upload10ms_fg_P$P" --size=$S --pool=5 --pinned --staged --wave-parts=64 --first-wave=4 --upload-ms=10 --foreground || exit 1
  run "staged_n5_whole_upload10ms_P$P" --size=$S --pool=5 --pinned --staged --upload-ms=10 || exit 1
  run "waves_n5_upload10ms_P$P" --size=$S --pool=5 --pinned --upload-ms=10 || exit 1
done
run "staged_n5_4files_P128" --size=$((128 * 10 * 1024 * 1024)) --pool=5 --pinned --staged --files=4 --wave-parts=32 || exit 1
