# round 4 ac: the multi-launch fused-rollout parity case, then more learning-curve seeds of the
# on-device trainer with fused rollouts (bench.py's train config, fp64 env): seeds 3 and 4 for 393 M
# env steps, seed 0 for 786 M (6000 iterations from scratch)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4ac
timeout -k 10 300 python -u -m pytest tests/test_gpu_rollout.py -m gpu -v -k "matches_env_replay" --timeout 200 --timeout-method thread > gpurun_out/r4ac/rollout_test.log 2>&1 || exit 2
for s in 3 4; do
  timeout -k 10 330 python -u tools/probes/gpu_learning_curve.py 3000 stand fp64 $s > gpurun_out/r4ac/lc_fp64_seed$s.log 2>&1 || exit 3
done
timeout -k 10 450 python -u tools/probes/gpu_learning_curve.py 6000 stand fp64 0 > gpurun_out/r4ac/lc_fp64_seed0_786M.log 2>&1 || exit 4
