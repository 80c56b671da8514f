# round 3b: per-phase cycles of the current fp64 / fp32 kernels (timing build, staggered mix)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/probes/gpu_timing.py fp64 staggered > gpurun_out/r3b_timing_fp64.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/probes/gpu_timing.py fp32 staggered > gpurun_out/r3b_timing_fp32.log 2>&1 || exit 2
