#!/bin/bash
# Round 6: the in-qsfs flush path against the loop it
# replaces, and where the staged binding's time goes.
#   - reference loop: DoMultiPartUpload with -m exactly as the reference runs it
#     (Acquire, ReadNoLoad, the reference's own md5(shared_ptr<iostream>) from
#     oracle/_ref, upload), sync (qsfs's File::Flush) and on a 5-thread executor;
#   - the staged binding (qsmd5::upload_parts_staged), auto and forced GPU, with
#     and without the upload loop's read-ahead;
#   - at -n 5, 128 and 512 x 10 MiB parts, uploads that return at once and 10 ms
#     uploads.
# QSMD5_TRACE=1: each qsmd5_hash_read call's phase times ride along ("traces").
# Every digest is checked against tests/golden/batch_10MiB.json.
# Output: gpurun_out/${OUT_NAME:-r06_flush_sweep}.jsonl, one line per case.
set -o pipefail
mkdir -p gpurun_out
OUT=gpurun_out/${OUT_NAME:-r06_flush_sweep}.jsonl
: > $OUT
H=tests/cpp/multipart_harness
run() {  # case-name, args...
  local name=$1; shift
  QSMD5_TRACE=1 timeout -k 10 300 env QSMD5_BACKEND=${BACKEND:-auto} $H --aligned "$@" \
    > gpurun_out/_one.json 2> gpurun_out/_one.err || { tail -5 gpurun_out/_one.err; return 1; }
  python3 - "$name" >> $OUT <<'PY'
import json, sys
r = json.load(open("gpurun_out/_one.json"))
gold = json.load(open("tests/golden/batch_10MiB.json"))["md5"]
r["case"] = sys.argv[1]
r["golden_ok"] = all(m == gold[:len(m)] for m in r["md5_files"])
for k in ("md5", "md5_files", "part_sizes"):
    r.pop(k, None)
r["traces"] = [json.loads(l.split("qsmd5 read trace: ", 1)[1]) for l in open("gpurun_out/_one.err")
               if "qsmd5 read trace: " in l]
print(json.dumps(r))
PY
  echo "$name $(python3 -c "import json;r=[json.loads(l) for l in open('$OUT')][-1];print(r['golden_ok'], r['wall_s_runs'], r['hash_s'])")" >&2
}
CASES=${CASES:-all}
for P in ${PARTS:-128 512}; do
  S=$((P * 10 * 1024 * 1024))
  if [[ $CASES == all || $CASES == *auto* ]]; then
    # the whole file as one pre-hash wave, auto vs forced GPU
    run "staged_whole_auto_P$P" --size=$S --pool=5 --pinned --staged --repeat=3 || exit 1
    BACKEND=gpu run "staged_whole_gpu_P$P" --size=$S --pool=5 --pinned --staged --repeat=3 || exit 1
  fi
  if [[ $CASES == all || $CASES == *ref* ]]; then
    for U in 0 10; do
      run "reference_sync_u${U}_P$P" --size=$S --pool=5 --reference-loop --upload-ms=$U || exit 1
      run "reference_async5_u${U}_P$P" --size=$S --pool=5 --reference-loop --async=5 --upload-ms=$U || exit 1
      run "staged_ramp_u${U}_P$P" --size=$S --pool=5 --pinned --staged --wave-parts=64 --first-wave=4 \
        --upload-ms=$U --repeat=2 || exit 1
      run "staged_ramp_noahead_u${U}_P$P" --size=$S --pool=5 --pinned --staged --wave-parts=64 --first-wave=4 \
        --upload-ms=$U --no-read-ahead --repeat=2 || exit 1
      run "staged_whole_u${U}_P$P" --size=$S --pool=5 --pinned --staged --upload-ms=$U --repeat=2 || exit 1
    done
  fi
  if [[ $CASES == all || $CASES == *sync* ]]; then
    # qsfs's default mode (qsSingleThread, Parser.cpp:286): File::Flush uploads
    # synchronously under the file's lock (File.cpp:619, 641-643), so the
    # binding runs without its helper thread (pipeline off: the whole file
    # pre-hashed on the flushing thread, no read-ahead)
    for U in 0 10; do
      run "staged_sync_u${U}_P$P" --size=$S --pool=5 --pinned --staged --no-pipeline --upload-ms=$U --repeat=2 || exit 1
    done
  fi
  if [[ $CASES == all || $CASES == *files* ]] && [[ $P == 128 ]]; then
    # four files flushed at once from four threads through one 5-buffer pool
    run "staged_4files_ramp_u0_P$P" --size=$S --pool=5 --pinned --staged --files=4 --wave-parts=32 --repeat=2 || exit 1
    run "staged_4files_whole_u0_P$P" --size=$S --pool=5 --pinned --staged --files=4 --repeat=2 || exit 1
    run "reference_sync_4files_u0_P$P" --size=$S --pool=5 --reference-loop --files=4 || exit 1
  fi
  if [[ $CASES == all || $CASES == *rate* ]]; then
    # the pre-hash's own rate with 1 and 4 readers, copy/kernel overlapped or
    # in one stream, over 2..4 staging regions; forced
    # GPU, uploads return at once
    for R in 1 4; do
      RP=""; [[ $R -gt 1 ]] && RP="--read-parallel"
      QSMD5_READ_THREADS=$R QSMD5_READ_OVERLAP=0 BACKEND=gpu run "prehash_readers${R}_overlap0_regions2_P$P" \
        --size=$S --pool=5 --pinned --staged --repeat=3 $RP || exit 1
      for G in 2 3 4; do
        QSMD5_READ_THREADS=$R QSMD5_READ_REGIONS=$G BACKEND=gpu run "prehash_readers${R}_overlap1_regions${G}_P$P" \
          --size=$S --pool=5 --pinned --staged --repeat=5 $RP || exit 1
      done
    done
  fi
done
echo "sweep done: $OUT" >&2
