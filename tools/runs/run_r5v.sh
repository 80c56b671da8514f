# round 5 v: staggered episode clocks as a PPO / HumanoidVecEnv option: the PPO GPU suite (incl. the
# learning regression test, now staggered) and the bench line (train leg staggered)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5v
timeout -k 10 600 python -u -m pytest tests/test_gpu_ppo.py -v -x --timeout 300 --timeout-method thread -p no:cacheprovider -s > gpurun_out/r5v/gputest.log 2>&1 || exit 3
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/r5v/bench.log 2>&1 || exit 4
