# multi-rank rehearsal on one GPU: 2 ranks (gloo backend for the timing reductions / all-reduce)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r2c
HSIM_BENCH_BACKEND=gloo timeout -k 10 300 python -u bench.py --gpus 2 --steps 10 --warmup 3 --no-episodes --no-configs --train-iters 1 --no-gae > gpurun_out/r2c/mr2.log 2>&1
