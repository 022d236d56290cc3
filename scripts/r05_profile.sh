#!/bin/bash
# scripts/r05_profile.sh -- round 5's rocprofv3 evidence: the stamped
# coalesced kernel (scripts/r05_stamps.sh), then scripts/profile_round.sh
# (kernel trace + stats of bench.py, FETCH_SIZE passes, the saturation lines).
# Summaries: python3 scripts/summarize_profiles.py r05.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
bash scripts/r05_stamps.sh || exit 1
cd "$R"
bash scripts/profile_round.sh
