# round 5 ag: colsum_pair's bias finish over 16 blocks (16 columns x 64 row phases), hs_dgrad_mask
# with 64-row workgroups above 16384 rows: parity, per-call timing (row blocks forced 2 / 4 / auto),
# A/B of the update's time per iteration, kernel trace of both paths
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5ag
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_ppo.py \
  -k "dgrad_mask or chain_node or relu_grad or deep_net" > gpurun_out/r5ag/tests.log 2>&1 || exit 2
HSIM_DG_RB=2 timeout -k 10 120 python tools/probes/gpu_dgrad_mask.py > gpurun_out/r5ag/micro_rb2.log 2>&1 || exit 3
HSIM_DG_RB=4 timeout -k 10 120 python tools/probes/gpu_dgrad_mask.py > gpurun_out/r5ag/micro_rb4.log 2>&1 || exit 3
timeout -k 10 120 python tools/probes/gpu_dgrad_mask.py > gpurun_out/r5ag/micro.log 2>&1 || exit 3
for r in 1 2; do
  timeout -k 10 300 python tools/probes/gpu_train_split.py 8 > gpurun_out/r5ag/chain_$r.log 2>&1 || exit 4
  timeout -k 10 300 python tools/probes/gpu_train_split.py 8 nochain > gpurun_out/r5ag/nochain_$r.log 2>&1 || exit 5
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5ag/prof_chain -o run -- python3 tools/probes/gpu_train_split.py 4 \
  > gpurun_out/r5ag/prof_chain.log 2>&1 || exit 6
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5ag/prof_nochain -o run -- python3 tools/probes/gpu_train_split.py 4 nochain \
  > gpurun_out/r5ag/prof_nochain.log 2>&1 || exit 7
