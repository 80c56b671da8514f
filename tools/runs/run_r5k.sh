# round 5 k: GAE as three launches for long rollouts (+ the fused MLP forward of r5j): GPU suites of
# PPO / rollout / GAE and the default bench line
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5k
timeout -k 10 600 python -u -m pytest tests/test_gpu_gae.py tests/test_gpu_ppo.py tests/test_gpu_rollout.py -v -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r5k/gputest.log 2>&1 || exit 3
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/r5k/bench.log 2>&1 || exit 5
