# round 4 d: the reference's own PPO hyperparameters (README.md:23-53), stand, fp64, 20 M env steps,
# 16 384 samples per rollout as 128 envs x 128 steps; seeds 0-2 as three processes on the one GPU
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4d
pids=()
for s in 0 1 2; do
  timeout -k 10 1080 python -u tools/probes/gpu_learning_curve_ref.py --seed $s --steps 20e6 --every 10 \
    > gpurun_out/r4d/lc_seed$s.log 2>&1 &
  pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait $p || rc=$?; done
exit $rc
