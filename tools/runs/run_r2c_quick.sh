# quick A/B loop: headline (fp64 staggered) + fp32 leg, no extra legs; contact/parity GPU tests
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r2c
timeout -k 10 300 python -u bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-rollout --no-gae --train-iters 0 --no-configs --no-episodes > gpurun_out/r2c/bench_quick.log 2>&1 || exit 3
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_contacts.py tests/test_gpu_pgs.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r2c/quick_tests.log 2>&1 || exit 1
