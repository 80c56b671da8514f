# round 2: rocprof evidence for the fp64 headline kernel (and the fp32 engine), then the summaries
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 bash profiles/collect.sh r2a fp64 > gpurun_out/collect_r2a.log 2>&1 || exit 1
timeout -k 10 900 bash profiles/collect.sh r2b fp32 > gpurun_out/collect_r2b.log 2>&1 || exit 2
