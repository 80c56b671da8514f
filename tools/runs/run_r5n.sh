# round 5 n: the PPO update's epoch graph as DOT (node kinds between the kernels)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5n
timeout -k 10 300 python tools/probes/gpu_graph_dump.py gpurun_out/r5n > gpurun_out/r5n/log.txt 2>&1 || exit 3
