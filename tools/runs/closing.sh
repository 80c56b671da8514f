# Closing evidence of a build: full GPU suite, the default bench line, rocprofv3 evidence of the headline
# kernel (stats + HBM + SQ passes) and of the train leg's fused rollout kernel, the instruction census, smoke.
#   gpurun --timeout 1200 -- 'bash tools/runs/closing.sh r6n'
# then: python profiles/summarize.py TAG fp64; python profiles/summarize_rollout.py TAG_rollout;
#       python tools/census_report.py TAG
TAG=${1:?usage: closing.sh TAG}
cd $GRAFT_REPO_ROOT
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gputest.log 2>&1
rc=$?
echo "pytest rc $rc" >> $O/gputest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit 3; fi
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || exit 4
bash profiles/collect.sh $TAG fp64 > $O/collect.log 2>&1 || exit 5
bash profiles/collect_rollout.sh ${TAG}_rollout > $O/collect_rollout.log 2>&1 || exit 6
bash profiles/census.sh $TAG > $O/census.log 2>&1 || exit 7
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 8
