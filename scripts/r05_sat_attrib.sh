#!/bin/bash
# scripts/r05_sat_attrib.sh -- round 5: where does the
# coalesced throughput kernel lose at 131072 x 64 KiB (60% of 8 TB/s) against
# 131072 x 256 KiB (69%) at the same 1.0003x traffic?
#   1. HIP-event medians over 131072 x {16,32,64,128,256} KiB (bench_configs
#      satsweep): t(L) = a + b*L splits a per-launch constant from the per-byte rate
#   2. the same under rocprofv3 --kernel-trace --stats (per-dispatch durations)
#   3. PMC passes at 64 and 256 KiB, one counter set per run: effective clock
#      (GRBM_GUI_ACTIVE / 8 XCDs / wall), mean wave lifetime against the
#      dispatch (SQ_WAVE_CYCLES / SQ_WAVES, quad-cycles), instructions per byte
#      (SQ_INSTS_VALU / SALU), issue vs wait (SQ_ACTIVE_INST_VALU, SQ_WAIT_INST_ANY)
# Raw outputs: gpurun_out/r05_sat/; summary: scripts/summarize_sat_attrib.py.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/r05_sat
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
export PYTHONUNBUFFERED=1
timeout -s KILL 60 rocprofv3 -L > "$OUT/counters.txt" 2>&1 || true
timeout -k 10 300 python3 "$R/bench_configs.py" --configs satsweep --reps 10 > "$OUT/satsweep.jsonl" \
  2> "$OUT/satsweep.err" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o sat -- \
  python3 "$R/bench_configs.py" --configs satsweep --reps 10 > "$OUT/trace.jsonl" 2> "$OUT/trace.err" || exit 1
pass() {  # name, config, counters...
  local name=$1 cfg=$2
  shift 2
  timeout -s KILL 150 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/pmc_$name" -o pmc -- \
    python3 "$R/bench_configs.py" --configs "$cfg" --reps 3 > "$OUT/pmc_$name.jsonl" 2> "$OUT/pmc_$name.err"
  echo "pass $name rc=$?" >> "$OUT/passes.log"
}
for cfg in sat64 sat256; do
  pass "${cfg}_a" $cfg GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES
  pass "${cfg}_b" $cfg SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY
done
find "$OUT" -name "*.csv" | sort
