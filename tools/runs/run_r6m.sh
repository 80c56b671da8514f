# round 6 m: per-item durations of the chunk queue at 4096 envs (timing build), for a claim-order study
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python tools/probes/gpu_timing.py fp64 staggered > gpurun_out/r6m_timing_4096.txt 2>&1 || exit 3
