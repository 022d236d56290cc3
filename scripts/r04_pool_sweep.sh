#!/bin/bash
# scripts/r04_pool_sweep.sh -- round 4, VERDICT r03 items 3 and 4, on the GPU box.
#
# Item 3: the qsfs transfer pool holds -n buffers of -b MiB (TransferManager.h:74-86,
# Drive.cpp:124).  multipart_harness uploads a 128 x 10 MiB file (every part golden)
# through pools of -n 5/16/32/64/128 buffers, pinned or pageable-and-registered, with
# QSMD5_BACKEND=auto, sync uploads of no network time (the hashing side alone), with
# and without the wave pipeline, the pool reused for a second pass (reported).
# Item 4: the same file with a simulated 10 ms per-part upload, pipelined or not.
# One JSON line per run in gpurun_out/r04_pool_sweep.jsonl.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
H=tests/cpp/multipart_harness
OUT=$O/r04_pool_sweep.jsonl
: > "$OUT"
MiB=$((1 << 20))
run() {  # label, args...
  local label=$1
  shift
  echo "== $label $*" >&2
  timeout -k 10 120 env QSMD5_BACKEND=auto "$H" "$@" > "$O/r04_one.json"
  python3 - "$label" "$O/r04_one.json" "$OUT" <<'EOF'
import json, sys
label, src, dst = sys.argv[1:4]
r = json.load(open(src))
gold = json.load(open("tests/golden/batch_10MiB.json"))["md5"]
r["golden_ok"] = all(m == gold[:r["parts"]] for m in r["md5_files"])
r["label"] = label
for k in ("md5", "md5_files", "part_sizes"):
    r.pop(k, None)
open(dst, "a").write(json.dumps(r) + "\n")
print(label, "waves", r["waves"], "gpu", r["gpu_waves"], "cpu", r["cpu_waves"], "widest", r["widest_wave"],
      "wall", r["wall_s_runs"], "golden", r["golden_ok"], flush=True)
EOF
}
for n in 5 16 32 64 128; do
  for kind in pinned register; do
    for pipe in on off; do
      extra=()
      [ "$pipe" = off ] && extra+=(--no-pipeline)
      run "pool${n}_${kind}_pipe_${pipe}" --aligned --size=$((128 * 10 * MiB)) --pool=$n --$kind \
        --repeat=2 "${extra[@]}"
    done
  done
done
for n in 16 64; do
  for pipe in on off; do
    extra=()
    [ "$pipe" = off ] && extra+=(--no-pipeline)
    run "upload10ms_pool${n}_pinned_pipe_${pipe}" --aligned --size=$((128 * 10 * MiB)) --pool=$n --pinned \
      --upload-ms=10 "${extra[@]}"
  done
done
run "files4_pool16_register_upload10ms" --aligned --size=$((64 * 10 * MiB)) --pool=16 --register --files=4 \
  --upload-ms=10
echo "pool sweep done: $OUT" >&2
