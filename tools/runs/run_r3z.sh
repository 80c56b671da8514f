# A/B: Cholesky DPP pivots (dpp), + next block's columns by DPP (dpp2), each with the normal-range sqrt (sf)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash profiles/ab.sh r3z mujocoposelearning_amd/libhsim.so mujocoposelearning_amd/libhsim_dpp.so mujocoposelearning_amd/libhsim_dpp2.so mujocoposelearning_amd/libhsim_dppsf.so mujocoposelearning_amd/libhsim_dpp2sf.so || exit 3
