# round 5 s: the fused MLP forward through the C ABI on padded strides
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5s
timeout -k 10 300 python -u -m pytest tests/test_gpu_ppo.py -k "mlp" -v -x --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r5s/gputest.log 2>&1 || exit 3
