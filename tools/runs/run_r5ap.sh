# round 5 ap: seeds 5 and 6 with the fused backward and with the module-by-module one
# (HS_NOCHAIN=1): bench train config, staggered clocks, 3000 iterations (393 M env steps), four runs
# side by side
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5ap
for s in 5 6; do
  timeout -k 10 1000 python -u tools/probes/gpu_learning_curve.py 3000 stand fp64 $s 32768 4 1 > gpurun_out/r5ap/seed${s}_chain.log 2>&1 &
  HS_NOCHAIN=1 timeout -k 10 1000 python -u tools/probes/gpu_learning_curve.py 3000 stand fp64 $s 32768 4 1 > gpurun_out/r5ap/seed${s}_nochain.log 2>&1 &
done
wait
