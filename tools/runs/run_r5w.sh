# round 5 w: staggered clocks with more Adam steps per sample: batch 8192 x 10 epochs (160 steps per
# rollout) and batch 4096 x 10 epochs (320), seeds 0 and 1, 800 iterations (105 M env steps) each,
# four runs side by side on the one GPU
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5w
for s in 0 1; do
  timeout -k 10 1080 python -u tools/probes/gpu_learning_curve.py 800 stand fp64 $s 8192 10 1 > gpurun_out/r5w/b8192_seed$s.log 2>&1 &
  timeout -k 10 1080 python -u tools/probes/gpu_learning_curve.py 800 stand fp64 $s 4096 10 1 > gpurun_out/r5w/b4096_seed$s.log 2>&1 &
done
wait
