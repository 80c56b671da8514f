# per-phase cycles of the r3k fp64 engine (timing build, staggered mix) + reward cost A/B
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/probes/gpu_timing.py fp64 staggered > gpurun_out/r3l_timing_fp64.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/probes/gpu_reward_cost_probe.py fp64 > gpurun_out/r3l_reward.log 2>&1 || exit 2
