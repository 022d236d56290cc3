#!/bin/bash
# scripts/r04_clock_probe.sh -- round 4: the clock the headline kernel runs at.
# MI355X_MICROARCH.md 'DVFS give-back': effective clock = GRBM_GUI_ACTIVE / 8
# (summed over the 8 XCDs) / kernel wall time, within 3 % of the in-kernel
# clock on dispatches of 10 ms or more.  One --pmc pass over a short bench.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/clock
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d "$OUT/pmc" -o pmc -- \
  python3 "$R/bench.py" --no-cpu-baseline --no-config5 --steps 5 --warmup 2 > "$OUT/bench.json" 2> "$OUT/bench.err"
timeout -s KILL 200 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d "$OUT/pmc_sat" -o pmc -- \
  python3 "$R/bench_configs.py" --configs sat --reps 1 > "$OUT/sat.jsonl" 2> "$OUT/sat.err"
find "$OUT" -name "*.csv" | sort
