# round 4 af: learning curves to 786 M env steps (6000 iterations) for the three seeds that had not
# stood by 393 M or were still climbing (0, 3, 4): bench.py's train config, fused rollouts, fp64 env
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4af
for s in 0 3 4; do
  timeout -k 10 380 python -u tools/probes/gpu_learning_curve.py 6000 stand fp64 $s > gpurun_out/r4af/lc_fp64_seed$s.log 2>&1 || exit 3
done
