# release/acquire hand-off: repeat the queue+wide bitwise test, then the full GPU suite
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for r in 1 2 3 4; do
  timeout -k 10 200 python -u -m pytest tests/test_gpu_queue.py -m gpu -q --timeout 150 --timeout-method thread 2>&1 | grep -E "AssertionError|passed|failed" >> gpurun_out/r3f.log
done
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/r3f_tests.log 2>&1
tail -3 gpurun_out/r3f_tests.log >> gpurun_out/r3f.log
