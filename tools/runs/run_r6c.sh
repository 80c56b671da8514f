# round 6 c: fused-rollout launch timing (hs_last_tape_ms) + train roofline; rollout-kernel rocprof evidence
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6c
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_ppo.py tests/test_gpu_rollout.py tests/test_gpu_tape.py -v --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?
echo "rc $rc" >> $O/tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit 3; fi
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || exit 4
bash profiles/collect_rollout.sh r6c_rollout || exit 5
