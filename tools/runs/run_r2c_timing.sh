# phase / wave-lifetime timing of the step kernel (diagnostic build), staggered mix
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r2c
timeout -k 10 200 python -u tools/probes/gpu_timing.py fp64 staggered > gpurun_out/r2c/timing_fp64.log 2>&1 || exit 2
timeout -k 10 200 python -u tools/probes/gpu_timing.py fp32 staggered > gpurun_out/r2c/timing_fp32.log 2>&1 || exit 3
