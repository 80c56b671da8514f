# round 6 a: device reward entry (hs_reward_eval) + numpy-order sums in the step kernel, warnings on
# the drop-in path: the new tests, the full GPU suite, the default bench line
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6a
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_reward_eval.py tests/test_gpu_dropin_warnings.py -v -s --timeout 120 --timeout-method thread -p no:cacheprovider > $O/new_tests.log 2>&1
echo "new rc $?" >> $O/new_tests.log
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gputest.log 2>&1
rc=$?
echo "pytest rc $rc" >> $O/gputest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit 3; fi
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || exit 4
