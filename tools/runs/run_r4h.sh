# round 4 h: final checkpoint -- GPU suite, smoke, default bench line, rocprof trace + PMC passes of
# the fp64 step kernel (profiles/collect.sh r4h), small-batch PPO update kernel trace
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4h
timeout -k 10 900 python -u -m pytest tests -m gpu -v --maxfail=8 --timeout 300 --timeout-method thread > gpurun_out/r4h/gputest.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/r4h/gputest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4h/smoke.log 2>&1 || exit 5
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r4h/bench.log 2>&1 || exit 6
bash profiles/collect.sh r4h fp64 > gpurun_out/collect_r4h.log 2>&1 || exit 7
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4h/upd -o upd -- python3 tools/probes/gpu_update_small.py 2 > gpurun_out/r4h/upd.log 2>&1 || exit 8
exit $rc
