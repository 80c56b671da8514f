# Multi-rank rehearsal of bench.py on a one-GPU box: 2 ranks over gloo sharing the GPU, short windows,
# every leg (the 8-GPU RCCL run is the driver's, never started here).
#   gpurun -- 'bash tools/runs/rehearse_2rank.sh r6l'
TAG=${1:?usage: rehearse_2rank.sh TAG}
cd $GRAFT_REPO_ROOT
O=gpurun_out/$TAG
mkdir -p $O
HSIM_BENCH_BACKEND=gloo timeout -k 10 900 python bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline --no-episodes --cpu-steps 100 > $O/bench_2rank_gloo.log 2>&1 || exit 4
