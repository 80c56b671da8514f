# round 6 j: each reward computes only the sum it reads -- A/B against round 5's butterfly sums (HS_REWARD_HSUM)
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6j
mkdir -p $O
L=$GRAFT_REPO_ROOT/mujocoposelearning_amd
B="python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-rollout --no-gae --train-iters 0 --no-configs --no-fp32 --no-episodes --no-tape --no-dropin"
for i in 1 2 3; do
  timeout -k 10 300 $B > $O/ab_def_$i.log 2>&1 || exit 3
  HSIM_LIB=$L/libhsim_hsum.so timeout -k 10 300 $B > $O/ab_hsum_$i.log 2>&1 || exit 4
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_reward_eval.py tests/test_gpu_parity.py -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
echo "rc $?" >> $O/tests.log
