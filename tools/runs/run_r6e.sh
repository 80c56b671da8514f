# round 6 e: Newton direction by 2-pivot Gauss-Jordan (gj_solve2) + the full Hessian pipelined: GPU suite,
# A/B of the headline window against 1-pivot GJ (libhsim_gj1.so) and the round-5 Cholesky (libhsim_chol.so),
# census, per-phase split at 4096 and 8 envs
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6e
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gputest.log 2>&1
rc=$?
echo "pytest rc $rc" >> $O/gputest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit 3; fi
B="python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-rollout --no-gae --train-iters 0 --no-configs --no-fp32 --no-episodes --no-tape --no-dropin"
L=$GRAFT_REPO_ROOT/mujocoposelearning_amd
for i in 1 2; do
  timeout -k 10 300 $B > $O/ab_gj2_$i.log 2>&1 || exit 4
  HSIM_LIB=$L/libhsim_gj1.so timeout -k 10 300 $B > $O/ab_gj1_$i.log 2>&1 || exit 5
  HSIM_LIB=$L/libhsim_chol.so timeout -k 10 300 $B > $O/ab_chol_$i.log 2>&1 || exit 6
done
bash profiles/census.sh r6e || exit 7
timeout -k 10 200 python tools/probes/gpu_timing.py fp64 staggered > $O/timing_4096.txt 2>&1 || exit 8
timeout -k 10 200 python tools/probes/gpu_timing.py fp64 n=8 > $O/timing_8.txt 2>&1 || exit 9
