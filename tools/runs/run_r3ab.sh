# Hessian rows two columns per scheduling group (fp64): GPU suite + headline A/B window + timing build
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3ab_tests.log 2>&1 || { tail -30 gpurun_out/r3ab_tests.log; exit 1; }
tail -2 gpurun_out/r3ab_tests.log
bash profiles/ab.sh r3ab mujocoposelearning_amd/libhsim.so || exit 2
timeout -k 10 200 python -u tools/probes/gpu_timing.py fp64 staggered > gpurun_out/r3ab_timing_fp64.log 2>&1 || exit 3
