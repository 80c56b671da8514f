# cost-ordered chunk-queue claims: queue parity tests, A/B auto (cost order) vs fixed_order, timing-build tail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_queue.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r3m_tests.log 2>&1 || exit 1
rm -f gpurun_out/r3m_ab.log
for r in 1 2; do
  for S in auto fixed_order; do
    timeout -k 10 200 python -u bench.py --steps 100 --warmup 5 --no-cpu-baseline --no-rollout --no-gae \
      --train-iters 0 --no-configs --no-episodes --no-fp32 --schedule $S > gpurun_out/r3m_tmp.json 2> gpurun_out/r3m_err.log || exit 2
    python -c "
import json; d=json.loads([l for l in open('gpurun_out/r3m_tmp.json') if l.startswith('{')][-1])
print('$S', round(d['value']/1e6,4), 'M', round(d['roofline']['kernel_ms_per_launch'],4), 'ms', d['sim_stats']['warnings'])" >> gpurun_out/r3m_ab.log
  done
done
cat gpurun_out/r3m_ab.log
timeout -k 10 200 python -u tools/probes/gpu_timing.py fp64 staggered > gpurun_out/r3m_timing_fp64.log 2>&1 || exit 3
