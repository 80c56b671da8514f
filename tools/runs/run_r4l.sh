# round 4 l (re-created container; r4g-r4j outputs were lost with it): (1) the reference's PPO
# hyperparameters (README.md:23-53), 128 envs x 128 steps (16 384 samples per rollout, as 8 x 2048) with
# staggered episode clocks, stand, fp64, 20 M env steps, seeds 0-2 in the background; (2) the GPU
# control fit on synthetic end keys (does a global search reach the basin at all?)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4l
pids=()
for s in 0 1 2; do
  timeout -k 10 1080 python -u tools/probes/gpu_learning_curve_ref.py --seed $s --steps 20e6 --every 10 --stagger \
    > gpurun_out/r4l/lc_seed$s.log 2>&1 &
  pids+=($!)
done
timeout -k 10 420 python -u tools/probes/gpu_trajfit.py --synthetic --intervals 56,90 --variants truth --pop 4096 --gens 3000 \
  > gpurun_out/r4l/synthetic.md 2> gpurun_out/r4l/synthetic.err
rc=0
for p in "${pids[@]}"; do wait $p || rc=$?; done
exit $rc
