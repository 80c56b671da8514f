# round 5 o: A/B of the Cholesky pivot block with both 1/sqrt chains side by side (second pivot
# from the block determinant) against the previous build (ab_libs/libhsim_base.so): fp64 parity
# tests on the new build, then the per-step sim-only leg alternating base / new, three rounds
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5o
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_queue.py tests/test_gpu_tape.py -v -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r5o/gputest.log 2>&1 || exit 3
B="python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-rollout --no-gae --train-iters 0 --no-configs --no-fp32 --no-episodes --no-dropin"
for r in 1 2 3; do
  HSIM_LIB=$GRAFT_REPO_ROOT/ab_libs/libhsim_base.so timeout -k 10 300 $B > gpurun_out/r5o/base_$r.log 2>&1 || exit 4
  timeout -k 10 300 $B > gpurun_out/r5o/new_$r.log 2>&1 || exit 5
done
