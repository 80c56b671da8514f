# round 5 a: GPU suite (new tests first) + default bench line
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5a
timeout -k 10 900 python -u -m pytest tests/test_gpu_tape.py tests/test_gpu_queue.py tests/test_gpu_env.py tests/test_gpu_ppo.py tests/test_gpu_rollout.py tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r5a/gputest.log 2>&1
rc=$?
echo "pytest rc $rc" >> gpurun_out/r5a/gputest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit 3; fi
timeout -k 10 500 python bench.py --steps 20 --warmup 5 > gpurun_out/r5a/bench.log 2>&1 || exit 4
