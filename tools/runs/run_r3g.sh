# round 3g: UC pool hand-off + epoch tags (t), + fp64 lookahead Cholesky (tla), + no MachineLICM
# (tla_nolicm): queue probe on tla, then A/B vs r3a (base)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
HSIM_LIB=mujocoposelearning_amd/libhsim_tla.so timeout -k 10 200 python -u tools/probes/gpu_queue_wide_probe.py > gpurun_out/r3g_probe.log 2>&1 || exit 1
bash profiles/ab.sh r3g mujocoposelearning_amd/libhsim_base.so mujocoposelearning_amd/libhsim_t.so mujocoposelearning_amd/libhsim_tla.so mujocoposelearning_amd/libhsim_tla_nolicm.so || exit 3
