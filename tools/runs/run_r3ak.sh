# product = straight-line contact aggregates + cubic fp64 reciprocal: GPU suite; fp64 window; fp32 A/B vs f32noag
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3ak_tests.log 2>&1 || { tail -30 gpurun_out/r3ak_tests.log; exit 1; }
tail -2 gpurun_out/r3ak_tests.log
bash profiles/ab.sh r3ak mujocoposelearning_amd/libhsim.so || exit 2
bash profiles/ab.sh r3ak32 mujocoposelearning_amd/libhsim.so mujocoposelearning_amd/libhsim_f32noag.so -- --precision fp32 || exit 3
