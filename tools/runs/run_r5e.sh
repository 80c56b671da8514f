# round 5 e: single-env queue units for small-batch tape launches / fused rollouts (configs[4]):
# the tape, rollout and queue tests, then the configs legs of the bench
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5e
timeout -k 10 600 python -u -m pytest tests/test_gpu_tape.py tests/test_gpu_rollout.py tests/test_gpu_queue.py -m gpu -v -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r5e/tests.log 2>&1 || exit 2
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-rollout --no-gae --train-iters 0 --no-fp32 --no-episodes --no-dropin > gpurun_out/r5e/bench.log 2>&1 || exit 3
