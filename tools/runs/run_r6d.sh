# round 6 d: Newton direction by Gauss-Jordan (gj_solve) instead of chol_rows + chol_solve: full GPU suite,
# A/B of the headline window against the Cholesky build (libhsim_chol.so, HS_NEWTON_CHOL), census
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6d
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gputest.log 2>&1
rc=$?
echo "pytest rc $rc" >> $O/gputest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit 3; fi
B="python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-rollout --no-gae --train-iters 0 --no-configs --no-fp32 --no-episodes --no-tape --no-dropin"
for i in 1 2; do
  timeout -k 10 300 $B > $O/ab_gj_$i.log 2>&1 || exit 4
  HSIM_LIB=$GRAFT_REPO_ROOT/mujocoposelearning_amd/libhsim_chol.so timeout -k 10 300 $B > $O/ab_chol_$i.log 2>&1 || exit 5
done
bash profiles/census.sh r6d || exit 6
# per-phase split: the configs[1] window and one env's critical path at the reference's n_envs = 8
timeout -k 10 200 python tools/probes/gpu_timing.py fp64 staggered > $O/timing_4096.txt 2>&1 || exit 7
timeout -k 10 200 python tools/probes/gpu_timing.py fp64 n=8 > $O/timing_8.txt 2>&1 || exit 8
