# round 2 (session 3): rocprofv3 evidence for the fp64 headline (chunk-queue schedule) and fp32 leg
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash profiles/collect.sh r2c fp64 > gpurun_out/collect_r2c.log 2>&1 || exit 1
bash profiles/collect.sh r2d fp32 > gpurun_out/collect_r2d.log 2>&1 || exit 2
