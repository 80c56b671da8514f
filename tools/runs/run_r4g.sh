# round 4 g: (1) the reference's own PPO hyperparameters (README.md:23-53), stand, fp64, 20 M env steps,
# 16 384 samples per rollout as 128 envs x 128 steps, seeds 0-2 as three background processes; (2) meanwhile
# the GPU control fit with long CMA-ES runs on synthetic end keys
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4g
pids=()
for s in 0 1 2; do
  timeout -k 10 1050 python -u tools/probes/gpu_learning_curve_ref.py --seed $s --steps 20e6 --every 10 \
    > gpurun_out/r4g/lc_seed$s.log 2>&1 &
  pids+=($!)
done
timeout -k 10 400 python -u tools/probes/gpu_trajfit.py --synthetic --intervals 56,90 --variants truth --pop 2048 --gens 5000 \
  > gpurun_out/r4g/synthetic.md 2> gpurun_out/r4g/synthetic.err
timeout -k 10 400 python -u tools/probes/gpu_trajfit.py --synthetic --intervals 56,90 --variants truth --pop 8192 --gens 2000 \
  > gpurun_out/r4g/synthetic8k.md 2> gpurun_out/r4g/synthetic8k.err
rc=0
for p in "${pids[@]}"; do wait $p || rc=$?; done
exit $rc
