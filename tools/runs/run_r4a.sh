# round 4 checkpoint a: full GPU suite after the ADVICE fixes (ctrl_stale, mid memset, UC pool cap,
# per-minibatch weights, subtree_com view)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4a
timeout -k 10 900 python -u -m pytest tests -m gpu -v --maxfail=8 --timeout 300 --timeout-method thread > gpurun_out/r4a/gputest.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/r4a/gputest.log
exit $rc
