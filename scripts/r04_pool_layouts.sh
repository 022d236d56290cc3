#!/bin/bash
# scripts/r04_pool_layouts.sh -- round 4: INTEGRATION.md §3's pool-layout table
# (512 x 10 MiB golden file through one wave) re-measured on the host-ordered
# staging pipeline: first pass and the pool reused, per layout.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
OUT=$O/r04_pool_layouts.jsonl
: > "$OUT"
MiB=$((1 << 20))
run() {
  local label=$1 envs=$2
  shift 2
  timeout -k 10 180 env QSMD5_BACKEND=gpu $envs tests/cpp/multipart_harness --aligned --size=$((512 * 10 * MiB)) \
    --pool=512 --repeat=3 --no-pipeline "$@" > "$O/r04_one.json"
  python3 - "$label" "$O/r04_one.json" "$OUT" <<'PY'
import json, sys
label, src, dst = sys.argv[1:4]
r = json.load(open(src))
gold = json.load(open("tests/golden/batch_10MiB.json"))["md5"]
r["golden_ok"] = r["md5"] == gold[:r["parts"]]
r["label"] = label
for k in ("md5", "md5_files", "part_sizes"):
    r.pop(k, None)
open(dst, "a").write(json.dumps(r) + "\n")
h = r["hash_s_runs"]
print("%-36s first %.1f GiB/s, reused %.1f GiB/s (hash only; register %.2f s) golden %s" % (
    label, 5.0 / h[0], 5.0 / min(h[1:]), r["register_s"], r["golden_ok"]), flush=True)
PY
}
run "slab pinned" "" --pinned --slab
run "slab pageable registered" "" --slab --register
run "separate pinned (gather kernel)" "" --pinned
run "separate pageable registered" "" --register
run "separate pageable" ""
run "slab pageable" "" --slab
run "separate pinned, QSMD5_GATHER=0" "QSMD5_GATHER=0" --pinned
