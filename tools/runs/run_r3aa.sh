# Cholesky pivots by DPP + normal-range sqrt now the product: GPU suite, then A/B fp64 (product vs
# direct 1/sqrt variant sf2 vs the round-3 kernel nodpp) and fp32 (product vs f32nodpp)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3aa_tests.log 2>&1 || { tail -30 gpurun_out/r3aa_tests.log; exit 1; }
tail -2 gpurun_out/r3aa_tests.log
bash profiles/ab.sh r3aa mujocoposelearning_amd/libhsim.so mujocoposelearning_amd/libhsim_sf2.so mujocoposelearning_amd/libhsim_nodpp.so || exit 2
bash profiles/ab.sh r3aa32 mujocoposelearning_amd/libhsim.so mujocoposelearning_amd/libhsim_f32nodpp.so -- --precision fp32 || exit 3
