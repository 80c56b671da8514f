cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/probes/gpu_timing.py fp64 staggered > gpurun_out/timing_fp64.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/probes/gpu_timing.py fp32 staggered > gpurun_out/timing_fp32.log 2>&1 || exit 2
timeout -k 10 200 python -u bench.py --envs 2048 --steps 20 --warmup 5 --no-cpu-baseline --no-rollout --no-gae --train-iters 0 --no-configs --no-episodes > gpurun_out/bench2048.log 2>&1 || exit 3
