cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --maxfail=8 --timeout 300 --timeout-method thread > gpurun_out/gputest.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/gputest.log
if [ $rc -eq 0 ] || [ $rc -eq 1 ]; then
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1
  echo "bench rc=$?" >> gpurun_out/bench.log
fi
