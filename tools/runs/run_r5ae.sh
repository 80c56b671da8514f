# round 5 ae: hs_dgrad_mask (input gradient + ReLU mask + bias first pass in one kernel) --
# parity tests, then A/B of the whole-net backward node on the update's time per iteration,
# alternating, two rounds, then a kernel trace of the chain path
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5ae
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_ppo.py \
  -k "dgrad_mask or chain_node or relu_grad or deep_net" > gpurun_out/r5ae/tests.log 2>&1 || exit 2
for r in 1 2; do
  timeout -k 10 300 python tools/probes/gpu_train_split.py 8 > gpurun_out/r5ae/chain_$r.log 2>&1 || exit 3
  timeout -k 10 300 python tools/probes/gpu_train_split.py 8 nochain > gpurun_out/r5ae/nochain_$r.log 2>&1 || exit 4
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5ae/prof -o run -- python3 tools/probes/gpu_train_split.py 4 \
  > gpurun_out/r5ae/prof.log 2>&1 || exit 5
