#!/bin/bash
# scripts/r06_profile.sh -- round 6's rocprofv3 evidence and the flush sweep on
# the final tree: scripts/profile_round.sh's passes (kernel trace + stats of
# bench.py, FETCH_SIZE of bench.py and of the calibration read, the saturation
# lines), one GRBM_GUI_ACTIVE pass of bench.py for the effective clock
# (scripts/summarize_clock.py), then scripts/r06_flush_sweep.sh.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
bash scripts/profile_round.sh || exit 1
OUT=$R/gpurun_out/clock
mkdir -p "$OUT"
(cd /tmp && TMPDIR=/tmp timeout -s KILL 150 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv \
  -d "$OUT/pmc" -o pmc -- python3 "$R/bench.py" --no-cpu-baseline --no-config5 --steps 5 --warmup 2 \
  > "$OUT/bench.json" 2> "$OUT/bench.err") || exit 1
python3 scripts/summarize_clock.py "$OUT/pmc/pmc_counter_collection.csv" \
  "bench.py --no-cpu-baseline --no-config5 --steps 5 --warmup 2 (headline, B=512 x 10 MiB)" \
  > "$R/gpurun_out/r06_effective_clock.log" || exit 1
OUT_NAME=r06_flush_sweep_tree timeout -k 10 900 bash scripts/r06_flush_sweep.sh 2> "$R/gpurun_out/r06_flush_sweep_tree.err"
