# round 5 z: staggered learning with a larger step size (lr 1e-3) and with more minibatches per
# epoch (batch 16384 x 4 epochs), seeds 0 and 1, 3000 iterations (393 M env steps), side by side
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5z
for s in 0 1; do
  timeout -k 10 1080 python -u tools/probes/gpu_learning_curve.py 3000 stand fp64 $s 32768 4 1 1e-3 > gpurun_out/r5z/lr1e-3_seed$s.log 2>&1 &
  timeout -k 10 1080 python -u tools/probes/gpu_learning_curve.py 3000 stand fp64 $s 16384 4 1 3e-4 > gpurun_out/r5z/b16384_seed$s.log 2>&1 &
done
wait
