cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/probes/gpu_pgs_probe2.py > gpurun_out/pgs_probe2.log 2>&1 || exit 1
