# round 5 an: learning after the fused backward, more seeds: seeds 3 and 4 with the fused backward,
# seed 1 with the module-by-module backward (HS_NOCHAIN=1) as the A/B for r5am's seed 1; bench
# train config, staggered clocks, 3000 iterations (393 M env steps), three runs side by side
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5an
for s in 3 4; do
  timeout -k 10 1000 python -u tools/probes/gpu_learning_curve.py 3000 stand fp64 $s 32768 4 1 > gpurun_out/r5an/seed$s.log 2>&1 &
done
HS_NOCHAIN=1 timeout -k 10 1000 python -u tools/probes/gpu_learning_curve.py 3000 stand fp64 1 32768 4 1 > gpurun_out/r5an/seed1_nochain.log 2>&1 &
wait
