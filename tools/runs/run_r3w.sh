# back-substitution block size per precision (fp64 1, fp32 2): GPU suite + A/B headline window
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3w_tests.log 2>&1 || { tail -30 gpurun_out/r3w_tests.log; exit 1; }
tail -2 gpurun_out/r3w_tests.log
bash profiles/ab.sh r3w mujocoposelearning_amd/libhsim.so || exit 2
bash profiles/ab.sh r3w32 mujocoposelearning_amd/libhsim.so -- --precision fp32 || exit 3
