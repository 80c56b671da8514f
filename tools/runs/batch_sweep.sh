# Sim-only headline window (fp64, staggered episode phases, per-step launches) at growing batches per
# GPU: 4096 (configs[1]), 8192, 16384, 32768 -- how the chunk queue's end-of-launch drain amortizes.
#   gpurun -- 'bash tools/runs/batch_sweep.sh r6t'
TAG=${1:?usage: batch_sweep.sh TAG}
cd $GRAFT_REPO_ROOT
O=gpurun_out/$TAG
mkdir -p $O
for n in 4096 8192 16384 32768; do
  timeout -k 10 400 python bench.py --envs $n --steps 20 --warmup 5 --no-cpu-baseline --no-rollout --no-gae --train-iters 0 --no-configs --no-fp32 --no-episodes --no-tape --no-dropin > $O/envs_$n.log 2>&1 || exit 3
done
grep -o '"value": [0-9.]*' $O/envs_*.log
