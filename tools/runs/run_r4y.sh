# round 4 y: learning curves of the on-device trainer with fused rollouts (fp64 env, bench.py's train
# config: 4096 envs x 32 steps, batch 32768, 4 epochs, lr 3e-4, MLP[256,256]), 3000 iterations = 393 M
# env steps per seed, seeds 0-2 one after another
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4y
for s in 0 1 2; do
  timeout -k 10 330 python -u tools/probes/gpu_learning_curve.py 3000 stand fp64 $s > gpurun_out/r4y/lc_fp64_seed$s.log 2>&1 || exit 3
done
