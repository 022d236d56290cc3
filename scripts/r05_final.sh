#!/bin/bash
# scripts/r05_final.sh TAG -- round 5's evidence on one MI355X for the tree as
# it stands: the full -m gpu suite, smoke(), the default bench line
# (scripts/r05_suite.sh TAG), then scripts/profile_round.sh's rocprofv3 passes.
# Summaries: python3 scripts/summarize_profiles.py r05.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
bash scripts/r05_suite.sh "${1:-final}" || exit 1
cd "$R"
bash scripts/profile_round.sh
cd "$R"
bash scripts/r05_staged_sweep.sh 2> "$R/gpurun_out/r05_staged_sweep.err"
