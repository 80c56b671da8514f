# A/B: map_vx contact operands read before the body loop (me) vs product
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash profiles/ab.sh r3ao mujocoposelearning_amd/libhsim.so mujocoposelearning_amd/libhsim_me.so || exit 2
