# round 5 t: learning curves with more gradient steps per sample than bench.py's train config:
# batch 8192 x 10 epochs (160 Adam steps per 131 072-sample rollout instead of 16), fp64 env,
# fused rollouts, seeds 0-2 side by side on the one GPU, 1500 iterations (197 M env steps) each
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5t
for s in 0 1 2; do
  timeout -k 10 1000 python -u tools/probes/gpu_learning_curve.py 1500 stand fp64 $s 8192 10 > gpurun_out/r5t/seed$s.log 2>&1 &
done
wait
