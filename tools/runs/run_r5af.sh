# round 5 af: hs_dgrad_mask rewritten (W transposed once per call for 16-byte B loads, the epilogue
# through LDS; the head kernel with the G tile in LDS): parity, per-call timing against the
# unfused path, A/B on the update's time per iteration, kernel trace of both paths
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5af
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_ppo.py \
  -k "dgrad_mask or chain_node or relu_grad or deep_net" > gpurun_out/r5af/tests.log 2>&1 || exit 2
timeout -k 10 120 python tools/probes/gpu_dgrad_mask.py > gpurun_out/r5af/micro.log 2>&1 || exit 3
for r in 1 2; do
  timeout -k 10 300 python tools/probes/gpu_train_split.py 8 > gpurun_out/r5af/chain_$r.log 2>&1 || exit 4
  timeout -k 10 300 python tools/probes/gpu_train_split.py 8 nochain > gpurun_out/r5af/nochain_$r.log 2>&1 || exit 5
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5af/prof_chain -o run -- python3 tools/probes/gpu_train_split.py 4 \
  > gpurun_out/r5af/prof_chain.log 2>&1 || exit 6
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5af/prof_nochain -o run -- python3 tools/probes/gpu_train_split.py 4 nochain \
  > gpurun_out/r5af/prof_nochain.log 2>&1 || exit 7
