# fp64 scheduler-strategy variants vs the product build
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash profiles/ab.sh r3j2 mujocoposelearning_amd/libhsim.so mujocoposelearning_amd/libhsim_iilp.so mujocoposelearning_amd/libhsim_iilplicm.so mujocoposelearning_amd/libhsim_iminreg.so mujocoposelearning_amd/libhsim_imaxocc.so mujocoposelearning_amd/libhsim_memcl.so || exit 3
