# round 4 s: cost of the fused rollout's in-kernel policy; configs legs with the fused collect
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4s
timeout -k 10 300 python -u tools/probes/gpu_rollout_cost.py > gpurun_out/r4s/cost.log 2>&1 || exit 2
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-episodes --train-iters 0 --no-fp32 --no-gae > gpurun_out/r4s/bench.log 2>&1 || exit 4
