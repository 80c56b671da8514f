# round 4 ad: end-of-round checkpoint -- GPU suite (incl. the multi-launch fused-rollout case), smoke,
# default bench line, rocprof trace + PMC passes of the fp64 step kernel (profiles/collect.sh r4ad),
# then two more learning-curve seeds (3, 4; bench.py's train config with fused rollouts, 393 M env steps)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4ad
timeout -k 10 900 python -u -m pytest tests -m gpu -v --maxfail=8 --timeout 300 --timeout-method thread > gpurun_out/r4ad/gputest.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/r4ad/gputest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4ad/smoke.log 2>&1 || exit 5
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r4ad/bench.log 2>&1 || exit 6
bash profiles/collect.sh r4ad fp64 > gpurun_out/collect_r4ad.log 2>&1 || exit 7
for s in 3 4; do
  timeout -k 10 330 python -u tools/probes/gpu_learning_curve.py 3000 stand fp64 $s > gpurun_out/r4ad/lc_fp64_seed$s.log 2>&1 || exit 8
done
exit $rc
