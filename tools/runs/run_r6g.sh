# round 6 g: default build (Cholesky) -- full bench line (drop-in sweep 8..4096, train roofline with the
# committed rollout profile), per-phase split at 4096 (staggered window) and at 8 envs
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6g
mkdir -p $O
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || exit 3
timeout -k 10 200 python tools/probes/gpu_timing.py fp64 staggered > $O/timing_4096.txt 2>&1 || exit 4
timeout -k 10 200 python tools/probes/gpu_timing.py fp64 n=8 > $O/timing_8.txt 2>&1 || exit 5
