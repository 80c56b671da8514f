# round 5 j: the fused MLP forward with its row-block threshold: PPO / rollout GPU suites and the
# default bench line (rollout leg now through two fused launches per step)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5j
timeout -k 10 600 python -u -m pytest tests/test_gpu_ppo.py tests/test_gpu_rollout.py -v -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r5j/gputest.log 2>&1 || exit 3
timeout -k 10 300 python tools/probes/gpu_mlp2_fwd.py > gpurun_out/r5j/mlp2_probe.log 2>&1 || exit 4
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/r5j/bench.log 2>&1 || exit 5
