# product (pipelined CRB + Hessian rows): GPU suite; fp32 A/B product vs the fp32 engine without the CRB pipelining
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3ah_tests.log 2>&1 || { tail -30 gpurun_out/r3ah_tests.log; exit 1; }
tail -2 gpurun_out/r3ah_tests.log
bash profiles/ab.sh r3ah32 mujocoposelearning_amd/libhsim.so mujocoposelearning_amd/libhsim_f32noca.so -- --precision fp32 || exit 3
