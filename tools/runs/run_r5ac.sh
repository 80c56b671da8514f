# round 5 ac: the minibatch loss without the entropy launches at ent_coef 0 and with one fused add:
# the PPO GPU suite and the train leg
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5ac
timeout -k 10 600 python -u -m pytest tests/test_gpu_ppo.py tests/test_gpu_rollout.py -v -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r5ac/gputest.log 2>&1 || exit 3
timeout -k 10 600 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-rollout --no-gae --no-configs --no-fp32 --no-episodes --no-tape --no-dropin --train-iters 6 > gpurun_out/r5ac/bench_train.log 2>&1 || exit 4
