#!/bin/bash
# scripts/r04_spin_thread_probe.sh -- round 4: which runtime pattern keeps a HIP
# thread busy during a GPU wave.  multipart_harness, 64 x 10 MiB golden file,
# pinned slab pool, waves of 8 parts forced onto the GPU, under staging variants.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
LOG=$O/r04_spin_thread_probe.log
: > "$LOG"
for v in "default" "QSMD5_COLUMN_BYTES=0" "QSMD5_COPY_STREAMS=1" "QSMD5_COLUMN_BYTES=0 QSMD5_COPY_STREAMS=1" "QSMD5_TRACE=1"; do
  envs=""
  [ "$v" != default ] && envs="$v"
  timeout -k 10 120 env QSMD5_BACKEND=gpu $envs tests/cpp/multipart_harness --aligned \
    --size=$((64 * 10485760)) --pool=8 --pinned --slab --no-pipeline --repeat=2 > "$O/r04_one.json" 2> "$O/r04_one.err"
  python3 - "$v" "$O/r04_one.json" "$O/r04_one.err" >> "$LOG" <<'PY'
import json, sys
v, src, err = sys.argv[1:4]
r = json.load(open(src))
gold = json.load(open("tests/golden/batch_10MiB.json"))["md5"]
print("%-45s wall %s cpu %s threads %s golden %s" % (v, r["wall_s_runs"], r["cpu_s_runs"], r["busy_threads"],
      r["md5"] == gold[:r["parts"]]))
tr = [l for l in open(err) if l.startswith("qsmd5 trace:")]
if tr:
    print("    " + "    ".join(tr[:2]).rstrip())
PY
done
cat "$LOG"
