# bisect the queue-vs-direct bitwise mismatch: lookahead+tags build vs + no-MachineLICM build
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T="tests/test_gpu_queue.py::test_queue_with_wide_tier_reruns_bitwise_equals_direct tests/test_gpu_env.py::test_chunk_queue_schedule_bitwise_equals_direct tests/test_gpu_queue.py::test_single_env_schedule_bitwise_equals_paired"
for L in libhsim_la.so libhsim.so; do
  HSIM_LIB=mujocoposelearning_amd/$L timeout -k 10 300 python -u -m pytest $T -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/r3d_$L.log 2>&1
  echo "$L rc=$?" >> gpurun_out/r3d_summary.log
done
cat gpurun_out/r3d_summary.log
