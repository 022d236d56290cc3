#!/bin/bash
# scripts/r05_slots.sh -- round 5: concurrent pull-driven batches (read slots).
# tests/test_gpu_read.py, then four files of 128 x 10 MiB flushed at once
# through one 5-buffer pool, pre-hash forced to the GPU (one batch per file)
# or routed (auto, waves of 32), with QSMD5_READ_SLOTS = 1, 2, 4.
# Output: gpurun_out/r05_slots.jsonl (+ the test log).
set -uo pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_read.py \
  > "$O/r05_gpu_read_tests.log" 2>&1 || exit 1
OUT=$O/r05_slots.jsonl
: > "$OUT"
H=tests/cpp/multipart_harness
S=$((128 * 10 * 1024 * 1024))
for slots in 1 2 4; do
  for mode in gpu auto; do
    extra=""
    [ $mode = auto ] && extra="--wave-parts=32"
    timeout -k 10 300 env QSMD5_BACKEND=$mode QSMD5_READ_SLOTS=$slots $H --aligned --repeat=2 --size=$S \
      --pool=5 --pinned --staged --files=4 $extra > "$O/_slot.json" || exit 1
    python3 - "$slots" "$mode" >> "$OUT" <<'PY'
import json, sys
r = json.load(open("gpurun_out/_slot.json"))
gold = json.load(open("tests/golden/batch_10MiB.json"))["md5"]
r["case"] = "4files_P128_%s_slots%s" % (sys.argv[2], sys.argv[1])
r["golden_ok"] = all(m == gold[:len(m)] for m in r["md5_files"])
for k in ("md5", "md5_files", "part_sizes"):
    r.pop(k, None)
print(json.dumps(r))
PY
    echo "slots $slots $mode done" >&2
  done
done
