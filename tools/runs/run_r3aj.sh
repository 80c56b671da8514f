# round-3 checkpoint r3aj (pipelined CRB/Hessian, Cholesky early reads): full GPU suite, smoke, bench,
# rocprof; then per-phase timing and A/B of the cubic reciprocal (r3) / straight-line aggregates (ag)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3aj
timeout -k 10 900 python -u -m pytest tests -m gpu -v --maxfail=8 --timeout 300 --timeout-method thread > gpurun_out/r3aj/gputest.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/r3aj/gputest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3aj/smoke.log 2>&1 || exit 5
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r3aj/bench.log 2>&1 || exit 6
bash profiles/collect.sh r3aj fp64 > gpurun_out/collect_r3aj.log 2>&1 || exit 7
timeout -k 10 300 python -u tools/probes/gpu_timing.py fp64 staggered > gpurun_out/r3aj_timing_fp64.txt 2>&1 || exit 8
bash profiles/ab.sh r3aj mujocoposelearning_amd/libhsim.so mujocoposelearning_amd/libhsim_r3.so mujocoposelearning_amd/libhsim_ag.so || exit 9
