cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for r in 1 2; do
echo "== cached mid, run $r" >> gpurun_out/r3e.log
timeout -k 10 200 python -u tools/probes/gpu_queue_wide_probe.py >> gpurun_out/r3e.log 2>&1
done
timeout -k 10 200 python -u -m pytest tests/test_gpu_queue.py -m gpu -q --timeout 150 --timeout-method thread 2>&1 | grep -E "AssertionError|passed|failed" >> gpurun_out/r3e.log
