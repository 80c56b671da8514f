# round 4 n: tape launches (hs_step_tape) -- determinism probe, GPU tests of the new path and the queue
# tests, then a bench with the tape legs
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4n
timeout -k 10 300 python -u tools/probes/gpu_tape_probe2.py > gpurun_out/r4n/probe2.log 2>&1 || exit 2
timeout -k 10 600 python -u -m pytest tests/test_gpu_tape.py tests/test_gpu_queue.py tests/test_gpu_env.py -v -x --timeout 240 --timeout-method thread > gpurun_out/r4n/gputest.log 2>&1 || exit 3
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-episodes --train-iters 0 --no-rollout > gpurun_out/r4n/bench.log 2>&1 || exit 4
