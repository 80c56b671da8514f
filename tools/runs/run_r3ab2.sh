# product = DPP pivots + direct fp64 1/sqrt (HS_SQRT_FAST 2): GPU suite, A/B vs sf1
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3ab2_tests.log 2>&1 || { tail -30 gpurun_out/r3ab2_tests.log; exit 1; }
tail -2 gpurun_out/r3ab2_tests.log
bash profiles/ab.sh r3ab2 mujocoposelearning_amd/libhsim.so mujocoposelearning_amd/libhsim_sf1.so || exit 2
