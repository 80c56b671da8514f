# round 5 q: two processes stepping queued 4096-env fp64 batches on one GPU at once
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5q
timeout -k 10 400 python -u -m pytest tests/test_gpu_concurrent.py -v -x --timeout 360 --timeout-method thread -p no:cacheprovider > gpurun_out/r5q/gputest.log 2>&1 || exit 3
