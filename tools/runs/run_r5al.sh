# round 5 al: (after the fused backward of each net, _MLPChainFn) bench.py's train config (batch 32768 x 4 epochs) with STAGGERED episode clocks, as the
# reference's 8 envs x 2048-step rollouts see every episode phase; fp64 env, fused rollouts, seeds
# 0-2 side by side, 2200 iterations (288 M env steps) each
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5al
for s in 0 1 2; do
  timeout -k 10 1000 python -u tools/probes/gpu_learning_curve.py 2200 stand fp64 $s 32768 4 1 > gpurun_out/r5al/seed$s.log 2>&1 &
done
wait
