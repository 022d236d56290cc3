cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --maxfail=3 --timeout 300 --timeout-method thread > gpurun_out/r02_gputest1.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -5 gpurun_out/r02_gputest1.log
exit $rc
