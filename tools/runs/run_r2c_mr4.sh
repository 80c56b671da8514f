# multi-rank rehearsal on one GPU: 4 ranks x 4096 envs (gloo for the timing reductions / PPO all-reduce)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r2c
HSIM_BENCH_BACKEND=gloo timeout -k 10 400 python -u bench.py --gpus 4 --steps 10 --warmup 3 --no-episodes --no-configs --train-iters 1 --no-gae --no-fp32 > gpurun_out/r2c/mr4.log 2>&1
