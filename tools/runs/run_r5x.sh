# round 5 x: staggered-clock learning curves: stand seeds 3 and 4, and the kneeling reward
# (robust_kneeling_reward, the reference's second result) seed 0; 3000 iterations (393 M env steps)
# each, side by side on the one GPU
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5x
for s in 3 4; do
  timeout -k 10 1000 python -u tools/probes/gpu_learning_curve.py 3000 stand fp64 $s 32768 4 1 > gpurun_out/r5x/stand_seed$s.log 2>&1 &
done
timeout -k 10 1000 python -u tools/probes/gpu_learning_curve.py 3000 kneeling fp64 0 32768 4 1 > gpurun_out/r5x/kneeling_seed0.log 2>&1 &
wait
