# round 6 n: closing build (final) -- full GPU suite, the default bench line, rocprofv3 evidence of the headline
# kernel (stats + HBM + SQ passes) and of the train leg's fused rollout kernel, the instruction census, smoke
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6n
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gputest.log 2>&1
rc=$?
echo "pytest rc $rc" >> $O/gputest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit 3; fi
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || exit 4
bash profiles/collect.sh r6n fp64 > $O/collect.log 2>&1 || exit 5
bash profiles/collect_rollout.sh r6n_rollout > $O/collect_rollout.log 2>&1 || exit 6
bash profiles/census.sh r6n > $O/census.log 2>&1 || exit 7
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 8
