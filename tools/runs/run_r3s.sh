# L D L' Newton factor (fp64): GPU suite
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3s_tests.log 2>&1 || { tail -30 gpurun_out/r3s_tests.log; exit 1; }
tail -3 gpurun_out/r3s_tests.log
