# product (Cholesky early reads) GPU suite; A/B: Hessian rows pipelined (ha), CRB rows pipelined (ca), both (haca)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3ag_tests.log 2>&1 || { tail -30 gpurun_out/r3ag_tests.log; exit 1; }
tail -2 gpurun_out/r3ag_tests.log
bash profiles/ab.sh r3ag mujocoposelearning_amd/libhsim.so mujocoposelearning_amd/libhsim_ha.so mujocoposelearning_amd/libhsim_ca.so mujocoposelearning_amd/libhsim_haca.so || exit 2
