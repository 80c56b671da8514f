# round 5 ab: A/B of the fp64 kernels compiled with -fassociative-math -fno-signed-zeros
# -fno-trapping-math (ab_libs/libhsim_assoc.so) against the closing build (ab_libs/libhsim_base.so):
# per-step sim-only leg alternating, three rounds; then the fp64 parity / queue / tape tests on the
# variant
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5ab
B="python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-rollout --no-gae --train-iters 0 --no-configs --no-fp32 --no-episodes --no-dropin"
for r in 1 2 3; do
  HSIM_LIB=$GRAFT_REPO_ROOT/ab_libs/libhsim_base.so timeout -k 10 300 $B > gpurun_out/r5ab/base_$r.log 2>&1 || exit 4
  HSIM_LIB=$GRAFT_REPO_ROOT/ab_libs/libhsim_assoc.so timeout -k 10 300 $B > gpurun_out/r5ab/assoc_$r.log 2>&1 || exit 5
done
HSIM_LIB=$GRAFT_REPO_ROOT/ab_libs/libhsim_assoc.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_queue.py tests/test_gpu_tape.py -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r5ab/gputest_assoc.log 2>&1
echo "rc $?" >> gpurun_out/r5ab/gputest_assoc.log
