#!/bin/bash
# scripts/r05_stamps.sh -- round 5: the coalesced kernel's per-wave start/end
# stamps (ubench stamps: shader cycles and the 100 MHz constant clock) at
# 131072 x {16, 64, 256} KiB: the clock the waves ran at vs the ramp/tail
# spread (PMC side: scripts/r05_sat_attrib.sh).
set -uo pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p "$R/gpurun_out"
cd "$R"
timeout -k 10 180 ubench/ubench_md5 stamps > gpurun_out/r05_stamps.jsonl 2> gpurun_out/r05_stamps.err
