# A/B fp32: Cholesky trailing-column reads issued with the pivot reads (fenced) vs product
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash profiles/ab.sh r3ap32 mujocoposelearning_amd/libhsim.so mujocoposelearning_amd/libhsim_f32early.so -- --precision fp32 || exit 2
