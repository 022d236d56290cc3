#!/bin/bash
# scripts/r02_gpu_suite.sh -- the round's GPU check, run through gpurun:
#   1. the -m gpu suite (parity tests through the C-ABI)
#   2. __graft_entry__.smoke()
#   3. bench.py (default: N=1, config 2, CPU baseline)
# Each step has its own time limit and the chain stops at the first failure.
# Usage: bash scripts/r02_gpu_suite.sh <tag> [pytest selection...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-run}; shift
SEL=${@:-tests}
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest $SEL -m gpu -v --maxfail=3 --timeout 300 \
  --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/${TAG}_pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/${TAG}_smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/${TAG}_bench.json
exit $rc
