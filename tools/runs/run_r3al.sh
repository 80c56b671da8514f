# A/B: per-contact LDS operands read in one batch in J'f and the Hessian contact terms (cf), + next contact's reads ahead (cfa)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash profiles/ab.sh r3al mujocoposelearning_amd/libhsim.so mujocoposelearning_amd/libhsim_cf.so mujocoposelearning_amd/libhsim_cfa.so || exit 2
