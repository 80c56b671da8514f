# round 3a: full GPU test suite (lockstep trainer, RCCL world-1, queue hand-off hook, single-env
# schedule), then the configs[4] schedule probe and a short headline bench
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r3a_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/probes/gpu_sched_probe.py --envs 1024 512 2048 > gpurun_out/r3a_sched_fp64.log 2>&1 || exit 2
timeout -k 10 300 python -u tools/probes/gpu_sched_probe.py --envs 1024 2048 --precision fp32 > gpurun_out/r3a_sched_fp32.log 2>&1 || exit 3
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-rollout --no-gae --train-iters 1 --no-episodes > gpurun_out/r3a_bench.log 2>&1 || exit 4
