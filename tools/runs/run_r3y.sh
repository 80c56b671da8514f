# A/B: Cholesky pivot block by DPP broadcast (dpp), two-accumulator M·v (mvs), both (dppmvs) vs product
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash profiles/ab.sh r3y mujocoposelearning_amd/libhsim.so mujocoposelearning_amd/libhsim_dpp.so mujocoposelearning_amd/libhsim_mvs.so mujocoposelearning_amd/libhsim_dppmvs.so || exit 3
