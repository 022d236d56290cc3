set -euo pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r03k
mkdir -p "$O"
cd /tmp
export TMPDIR=/tmp
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
timeout -k 10 300 "$R/ubench/ubench_md5" attrib > "$O/attrib.log" 2>&1
timeout -k 10 120 "$R/ubench/ubench_md5" chaincost > "$O/chaincost.log" 2>&1
timeout -s KILL 200 rocprofv3 --pmc $C --output-format csv -d "$O/pmc_bench" -o pmc -- \
  python3 "$R/bench.py" --no-cpu-baseline --no-config5 --steps 2 --warmup 1 > "$O/pmc_bench.json" 2> "$O/pmc_bench.err"
timeout -s KILL 200 rocprofv3 --pmc $C --output-format csv -d "$O/pmc_attrib" -o pmc -- \
  "$R/ubench/ubench_md5" attrib > "$O/pmc_attrib.log" 2>&1
timeout -s KILL 200 rocprofv3 --pmc $C --output-format csv -d "$O/pmc_chain" -o pmc -- \
  "$R/ubench/ubench_md5" chaincost > "$O/pmc_chain.log" 2>&1
find "$O" -name "*.csv" | sort
