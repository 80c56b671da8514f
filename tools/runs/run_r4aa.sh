# round 4 aa: fused rollouts under a world-2 trainer (gloo, two ranks on one GPU)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4aa
timeout -k 10 400 python -u -m pytest tests/test_gpu_rollout.py -v -k multi_rank --timeout 300 --timeout-method thread > gpurun_out/r4aa/gputest.log 2>&1
