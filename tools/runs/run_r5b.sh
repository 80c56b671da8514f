# round 5 b: the fixed env test + the learning regression test with its numbers, the drop-in bench leg
# with the native info builder, then rocprofv3 evidence of the closing kernel -- per-step fp64
# launch (trace + stats, FETCH / WRITE passes, two SQ passes: profiles/collect.sh), the tape launch
# (collect_tape.sh), the rollout / train legs (kernel trace), and the timing build's per-phase
# split of the fp64 substep
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5b
timeout -k 10 300 python -u -m pytest tests/test_gpu_env.py tests/test_gpu_ppo.py -m gpu -v -s --timeout 200 --timeout-method thread -p no:cacheprovider -k "determinism or step_wait or stand_task" > gpurun_out/r5b/tests.log 2>&1 || exit 2
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-rollout --no-gae --train-iters 0 --no-configs --no-fp32 --no-episodes --no-tape > gpurun_out/r5b/dropin.log 2>&1 || exit 3
bash profiles/collect.sh r5b fp64 > gpurun_out/r5b/collect.log 2>&1 || exit 4
bash profiles/collect_tape.sh r5bt > gpurun_out/r5b/collect_tape.log 2>&1 || exit 5
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5b/roll -o trace -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-configs --no-fp32 --no-episodes --no-tape --no-gae --no-dropin --train-iters 3 > gpurun_out/r5b/roll_bench.log 2>&1 || exit 6
timeout -k 10 300 python3 tools/probes/gpu_timing.py fp64 staggered > gpurun_out/r5b/timing_fp64.txt 2>&1 || exit 7
