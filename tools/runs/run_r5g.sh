# round 5 g: closing-HEAD rocprofv3 evidence for the per-step fp64 kernel (kernel trace + stats,
# FETCH_SIZE / WRITE_SIZE passes, two SQ passes); summarized by profiles/summarize.py r5g fp64
cd $GRAFT_REPO_ROOT
bash profiles/collect.sh r5g fp64 > gpurun_out/r5g_collect.log 2>&1 || exit 3
