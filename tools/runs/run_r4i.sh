# round 4 i: (1) reference PPO hyperparameters (README.md:23-53), 128 envs x 128 steps with the envs'
# episode clocks staggered (every rollout holds every episode phase, as 8 envs x 2048 steps do), stand,
# fp64, 20 M steps, seeds 0-2 in the background; (2) the GPU control fit (CMA mean kept in the box):
# synthetic check, then recorded keys with the truth model and two wrong variants
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4i
pids=()
for s in 0 1 2; do
  timeout -k 10 1060 python -u tools/probes/gpu_learning_curve_ref.py --seed $s --steps 20e6 --every 10 --stagger \
    > gpurun_out/r4i/lc_seed$s.log 2>&1 &
  pids+=($!)
done
timeout -k 10 300 python -u tools/probes/gpu_trajfit.py --synthetic --intervals 56,90 --variants truth --pop 4096 --gens 3000 \
  > gpurun_out/r4i/synthetic.md 2> gpurun_out/r4i/synthetic.err
timeout -k 10 500 python -u tools/probes/gpu_trajfit.py --intervals 56,90 --variants truth,armature_zero,friction_07 --pop 4096 --gens 3000 \
  > gpurun_out/r4i/real.md 2> gpurun_out/r4i/real.err
rc=0
for p in "${pids[@]}"; do wait $p || rc=$?; done
exit $rc
