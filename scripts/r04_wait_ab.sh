#!/bin/bash
# scripts/r04_wait_ab.sh -- round 4: host CPU time of a synchronous GPU batch,
# spinning (hipStreamSynchronize) against sleeping (hipEventBlockingSync event),
# and what the switch costs small calls.  multipart_harness, 256 x 10 MiB golden
# file, pinned slab pool, GPU forced, waves of 8 / 64 / 256 parts; then
# ubench/small_call_latency.py under each mode.  Output: gpurun_out/r04_wait_ab.log
set -euo pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
LOG=$O/r04_wait_ab.log
: > "$LOG"
MiB=$((1 << 20))
for n in 8 64 256; do
  for w in spin block poll; do
    timeout -k 10 180 env QSMD5_BACKEND=gpu QSMD5_WAIT=$w tests/cpp/multipart_harness --aligned \
      --size=$((256 * 10 * MiB)) --pool=$n --pinned --slab --repeat=2 --no-pipeline > "$O/r04_one.json"
    python3 - "$n" "$w" "$O/r04_one.json" >> "$LOG" <<'EOF'
import json, sys
n, w, src = sys.argv[1:4]
r = json.load(open(src))
gold = json.load(open("tests/golden/batch_10MiB.json"))["md5"]
ok = r["md5"] == gold[:r["parts"]]
print("wave %3s parts  wait=%-5s  wall %.3f s  cpu %.3f s  (%.2f GiB/s; cpu per wall %.2f)  golden %s" % (
    n, w, r["wall_s_runs"][-1], r["cpu_s_runs"][-1], r["size"] / 2.0 ** 30 / r["wall_s_runs"][-1],
    r["cpu_s_runs"][-1] / r["wall_s_runs"][-1], ok), flush=True)
print("    threads still alive with > 50 ms of CPU (both passes):", r["busy_threads"], flush=True)
EOF
    tail -2 "$LOG"
  done
done
for w in spin poll; do
  echo "small calls, QSMD5_WAIT=$w" >> "$LOG"
  timeout -k 10 120 env QSMD5_BACKEND=gpu QSMD5_WAIT=$w python3 ubench/small_call_latency.py >> "$LOG" 2>&1
done
cat "$LOG"
