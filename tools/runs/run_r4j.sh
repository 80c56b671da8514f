# round 4 j: (1) the reference's config.py hyperparameters (README.md:154; lr 3e-4, batch 256,
# 20 epochs, ent 0, MLP[64,64], 5 M steps), stand, fp64, 128 envs x 128 steps, staggered episode
# clocks, seeds 0-2 in the background; (2) final checkpoint: GPU suite, smoke, bench, rocprof of the
# fp64 step kernel (collect.sh r4j), small-batch update kernel trace
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4j
pids=()
for s in 0 1 2; do
  timeout -k 10 700 python -u tools/probes/gpu_learning_curve_ref.py --config configpy --seed $s --steps 5e6 --every 10 --stagger \
    > gpurun_out/r4j/lc_cfg_seed$s.log 2>&1 &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p; done
timeout -k 10 900 python -u -m pytest tests -m gpu -v --maxfail=8 --timeout 300 --timeout-method thread > gpurun_out/r4j/gputest.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/r4j/gputest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4j/smoke.log 2>&1 || exit 5
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r4j/bench.log 2>&1 || exit 6
bash profiles/collect.sh r4j fp64 > gpurun_out/collect_r4j.log 2>&1 || exit 7
exit $rc
