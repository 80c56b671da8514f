# A/B: fp64 Cholesky pivot clamped before the DPP broadcast (pc), + trailing-column reads issued before the pivot math (early)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash profiles/ab.sh r3af mujocoposelearning_amd/libhsim.so mujocoposelearning_amd/libhsim_pc.so mujocoposelearning_amd/libhsim_early.so || exit 2
