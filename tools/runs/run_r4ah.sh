# round 4 ah: closing check at HEAD -- full GPU suite, smoke, default bench line
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4ah
timeout -k 10 900 python -u -m pytest tests -m gpu -v --maxfail=8 --timeout 300 --timeout-method thread > gpurun_out/r4ah/gputest.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/r4ah/gputest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4ah/smoke.log 2>&1 || exit 5
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r4ah/bench.log 2>&1 || exit 6
exit $rc
