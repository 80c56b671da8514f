# round 5 aq: closing build (in-context chain test, depth-parametrized chain test): the full GPU suite and the default bench line
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5aq
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r5aq/gputest.log 2>&1
rc=$?
echo "pytest rc $rc" >> gpurun_out/r5aq/gputest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit 3; fi
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/r5aq/bench.log 2>&1 || exit 4
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5aq/smoke.log 2>&1 || exit 5
