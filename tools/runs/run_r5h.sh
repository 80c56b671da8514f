# round 5 h: the fused policy-MLP forward rewritten (nn.Linear [out][in] weights, 16-byte weight
# loads streamed into a register ring, 8 waves per 16 rows): its tests, the rollout / PPO suites,
# the timing probe and the default bench line
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5h
timeout -k 10 600 python -u -m pytest tests/test_gpu_ppo.py tests/test_gpu_rollout.py -v -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r5h/gputest.log 2>&1 || exit 3
timeout -k 10 300 python tools/probes/gpu_mlp2_fwd.py > gpurun_out/r5h/mlp2_probe.log 2>&1 || exit 4
timeout -k 10 500 python bench.py --steps 20 --warmup 5 --no-dropin --no-configs --no-episodes > gpurun_out/r5h/bench.log 2>&1 || exit 5
