# A/B: pipelined Hessian rows with 3 (hg3) / 4 (hg4) columns per group vs 2 (product)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash profiles/ab.sh r3an mujocoposelearning_amd/libhsim.so mujocoposelearning_amd/libhsim_hg3.so mujocoposelearning_amd/libhsim_hg4.so || exit 2
