# round 4 z: fused rollout full-state case, PGS tape case
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4z
timeout -k 10 600 python -u -m pytest tests/test_gpu_rollout.py tests/test_gpu_tape.py -v --timeout 240 --timeout-method thread > gpurun_out/r4z/gputest.log 2>&1
