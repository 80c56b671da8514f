# round 3h: epoch tags + UC pool (t) vs + no MachineLICM (t_nolicm), fp64 and fp32, vs r3a (base)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash profiles/ab.sh r3h mujocoposelearning_amd/libhsim_base.so mujocoposelearning_amd/libhsim_t.so mujocoposelearning_amd/libhsim_t_nolicm.so || exit 3
bash profiles/ab.sh r3h32 mujocoposelearning_amd/libhsim_t.so mujocoposelearning_amd/libhsim_t_nolicm.so -- --precision fp32 || exit 4
