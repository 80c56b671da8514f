# round 2 quick loop: GPU parity tests of the step kernel (Newton + PGS), phase timing (fp64 / fp32,
# staggered mix), short headline bench, PGS cap probe
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_env.py tests/test_gpu_pgs.py tests/test_gpu_contacts.py tests/test_reference_pin.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/quick_tests.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/probes/gpu_timing.py fp64 staggered > gpurun_out/timing_fp64.log 2>&1 || exit 2
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-rollout --no-gae --train-iters 0 --no-configs --no-episodes > gpurun_out/bench_quick.log 2>&1 || exit 3
timeout -k 10 400 python -u tools/probes/gpu_pgs_probe2.py > gpurun_out/pgs_probe2.log 2>&1 || exit 4
