# round 4 r: fused PPO rollouts (hs_rollout) -- GPU tests of the new path, the PPO / tape / queue
# suites, then a bench with the collect_rollouts legs
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4r
timeout -k 10 600 python -u -m pytest tests/test_gpu_rollout.py tests/test_gpu_ppo.py tests/test_gpu_tape.py -v -x --timeout 240 --timeout-method thread > gpurun_out/r4r/gputest.log 2>&1 || exit 3
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-episodes --no-configs > gpurun_out/r4r/bench.log 2>&1 || exit 4
