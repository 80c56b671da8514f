# final round-3 checkpoint r3am (+ contact loops flat / ahead): full GPU suite, smoke, bench, rocprof,
# fp32 A/B of the contact-loop change, SURVEY 8(d) protocol (fp64, fp32), parity report
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3am
timeout -k 10 900 python -u -m pytest tests -m gpu -v --maxfail=8 --timeout 300 --timeout-method thread > gpurun_out/r3am/gputest.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/r3am/gputest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3am/smoke.log 2>&1 || exit 5
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r3am/bench.log 2>&1 || exit 6
bash profiles/collect.sh r3am fp64 > gpurun_out/collect_r3am.log 2>&1 || exit 7
bash profiles/ab.sh r3am32 mujocoposelearning_amd/libhsim.so mujocoposelearning_amd/libhsim_f32nocf.so -- --precision fp32 || exit 8
timeout -k 10 500 python -u bench.py --protocol --precision fp64 > gpurun_out/r3am/protocol_fp64.log 2>&1 || exit 9
timeout -k 10 400 python -u bench.py --protocol --precision fp32 > gpurun_out/r3am/protocol_fp32.log 2>&1 || exit 10
timeout -k 10 600 python -u tools/probes/parity_report.py > gpurun_out/r3am/parity_report.md 2> gpurun_out/r3am/parity_report.err || exit 11
