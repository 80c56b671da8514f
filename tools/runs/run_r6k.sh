# round 6 k: hs_reward (the device reward code on a batch's own buffers) -- reward tests
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6k
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_reward_eval.py tests/test_gpu_dropin_warnings.py -v --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
echo "rc $?" >> $O/tests.log
