# round 4 ab: free-running stream groups (2 / 4) for the fp64 sim-only per-step leg
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4ab
for g in 2 4; do
  timeout -k 10 300 python -u bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-rollout --no-gae --train-iters 0 --no-configs --no-fp32 --no-episodes --no-tape --free-groups $g > gpurun_out/r4ab/bench_g$g.log 2>&1 || exit 3
done
