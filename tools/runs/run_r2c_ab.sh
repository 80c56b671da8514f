# A/B: libhsim_base.so (before) vs libhsim.so (after), alternating, headline + fp32 legs only
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
B="python -u bench.py --steps 100 --warmup 5 --no-cpu-baseline --no-rollout --no-gae --train-iters 0 --no-configs --no-episodes"
for r in 1 2; do
  HSIM_LIB=$PWD/mujocoposelearning_amd/libhsim_base.so timeout -k 10 200 $B > gpurun_out/ab/base_$r.log 2>&1 || exit 1
  timeout -k 10 200 $B > gpurun_out/ab/new_$r.log 2>&1 || exit 2
done
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pgs.py tests/test_gpu_contacts.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/ab/tests.log 2>&1 || exit 3
