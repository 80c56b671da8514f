# round 5 ad: A/B of the value head's input gradient (broadcast multiply vs K = 1 mm) on the
# update's time per iteration, alternating, two rounds
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5ad
for r in 1 2; do
  timeout -k 10 300 python tools/probes/gpu_train_split.py 8 > gpurun_out/r5ad/mul_$r.log 2>&1 || exit 3
  timeout -k 10 300 python tools/probes/gpu_train_split.py 8 mm > gpurun_out/r5ad/mm_$r.log 2>&1 || exit 4
done
