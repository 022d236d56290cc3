#!/bin/bash
# scripts/profile_round.sh -- collect a round's rocprofv3 evidence on the GPU box
# (run through gpurun; nothing here runs in the build container).
#   1. kernel trace + stats of the headline command (python3 bench.py)
#   2. FETCH_SIZE of bench.py in its own pass (no trace domains with --pmc)
#   3. FETCH_SIZE calibration: ubench k_stream_read, 4 GiB coalesced read
#      (MI355X_MICROARCH.md: gfx950 FETCH_SIZE tallies 128-B requests at 64 B)
#   4. kernel trace + stats and FETCH_SIZE of the saturation lines
# Raw outputs land in gpurun_out/prof/; summaries are copied into profiles/.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/prof
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/bench" -o bench -- \
  python3 "$R/bench.py" > "$OUT/bench.json" 2> "$OUT/bench.err"
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_bench" -o pmc -- \
  python3 "$R/bench.py" --no-cpu-baseline --no-config5 --steps 2 --warmup 1 > "$OUT/pmc_bench.json" 2> "$OUT/pmc_bench.err"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_calib" -o pmc -- \
  "$R/ubench/ubench_md5" calib > "$OUT/pmc_calib.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/sat" -o sat -- \
  python3 "$R/bench_configs.py" --configs sat > "$OUT/sat.jsonl" 2> "$OUT/sat.err"
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_sat" -o pmc -- \
  python3 "$R/bench_configs.py" --configs sat --reps 1 > "$OUT/pmc_sat.jsonl" 2> "$OUT/pmc_sat.err"
find "$OUT" -name "*.csv" | sort
