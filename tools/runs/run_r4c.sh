# round 4 checkpoint c: GPU suite (probe path fix, whole-epoch update graph), fp32 event trace,
# reference-hyperparameter learning run timing
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4c
timeout -k 10 900 python -u -m pytest tests -m gpu -v --maxfail=8 --timeout 300 --timeout-method thread > gpurun_out/r4c/gputest.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/r4c/gputest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/probes/gpu_fp32_events.py > gpurun_out/r4c/fp32_events.md 2> gpurun_out/r4c/fp32_events.err || exit 5
timeout -k 10 300 python -u tools/probes/gpu_learning_curve_ref.py --seed 0 --steps 0.5e6 --every 5 > gpurun_out/r4c/lc_timing.log 2>&1 || exit 6

timeout -k 10 300 python -u tools/probes/gpu_timing.py fp64 staggered > gpurun_out/r4c/timing_fp64.txt 2>&1 || exit 7
exit $rc
