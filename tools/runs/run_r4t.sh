# round 4 t: fused rollout with the two-envs-per-lane policy layout: tests + cost probe
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4t
timeout -k 10 400 python -u -m pytest tests/test_gpu_rollout.py -v -x --timeout 240 --timeout-method thread > gpurun_out/r4t/gputest.log 2>&1 || exit 3
timeout -k 10 300 python -u tools/probes/gpu_rollout_cost.py > gpurun_out/r4t/cost.log 2>&1 || exit 2
