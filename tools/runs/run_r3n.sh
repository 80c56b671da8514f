# incremental Newton factor (fp64): GPU suite, A/B vs HSIM_NEWTON_REBUILD=1, timing build
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3n_tests.log 2>&1 || { tail -30 gpurun_out/r3n_tests.log; exit 1; }
tail -3 gpurun_out/r3n_tests.log
rm -f gpurun_out/r3n_ab.log
for r in 1 2; do
  for R in 0 1; do
    HSIM_NEWTON_REBUILD=$R timeout -k 10 200 python -u bench.py --steps 100 --warmup 5 --no-cpu-baseline --no-rollout --no-gae \
      --train-iters 0 --no-configs --no-episodes --no-fp32 > gpurun_out/r3n_tmp.json 2> gpurun_out/r3n_err.log || exit 2
    python -c "
import json; d=json.loads([l for l in open('gpurun_out/r3n_tmp.json') if l.startswith('{')][-1])
print('rebuild=$R', round(d['value']/1e6,4), 'M', round(d['roofline']['kernel_ms_per_launch'],4), 'ms', d['sim_stats']['warnings'], d['sim_stats'].get('mean_newton_iters'))" >> gpurun_out/r3n_ab.log
  done
done
cat gpurun_out/r3n_ab.log
timeout -k 10 200 python -u tools/probes/gpu_timing.py fp64 staggered > gpurun_out/r3n_timing_fp64.log 2>&1 || exit 3
