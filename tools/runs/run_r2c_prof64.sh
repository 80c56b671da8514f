cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash profiles/collect.sh r2c fp64 > gpurun_out/collect_r2c.log 2>&1 || exit 1
