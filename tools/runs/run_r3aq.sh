# product with the fp32 Cholesky early reads: GPU suite + smoke
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3aq_tests.log 2>&1 || { tail -30 gpurun_out/r3aq_tests.log; exit 1; }
tail -2 gpurun_out/r3aq_tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3aq_smoke.log 2>&1 || exit 5
tail -1 gpurun_out/r3aq_smoke.log
