# A/B: column-oriented back substitution through LDS (bl2 / f32bl), set-bit sums with loads one bit ahead (ba2 / f32ba)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash profiles/ab.sh r3ac mujocoposelearning_amd/libhsim.so mujocoposelearning_amd/libhsim_bl2.so mujocoposelearning_amd/libhsim_ba2.so || exit 2
bash profiles/ab.sh r3ac32 mujocoposelearning_amd/libhsim.so mujocoposelearning_amd/libhsim_f32bl.so mujocoposelearning_amd/libhsim_f32ba.so -- --precision fp32 || exit 3
