# round 2 (session 3, final kernel: permuted chunk queue): rocprofv3 evidence for the fp64 headline
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash profiles/collect.sh r2e fp64 > gpurun_out/collect_r2e.log 2>&1 || exit 1
