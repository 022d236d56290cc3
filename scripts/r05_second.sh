#!/bin/bash
# scripts/r05_second.sh -- round 5, second GPU call: the saturation attribution
# (scripts/r05_sat_attrib.sh), the staged sweep with the wave ramp, and the
# route sweep on the fixed lane pricing.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
bash scripts/r05_sat_attrib.sh > "$O/r05_sat_attrib.out" 2>&1 || exit 1
cd "$R"
bash scripts/r05_staged_sweep.sh 2> "$O/r05_staged_sweep.err" || exit 1
bash scripts/r05_route_sweep.sh > "$O/r05_route_sweep.out" 2> "$O/r05_route_sweep.err"
