# round 6 f: Cholesky lookahead (libhsim_la.so, HS_CHOL_LOOKAHEAD; must be bitwise the default) vs the
# default build, and the Gauss-Jordan build again (libhsim_gj.so) -- headline window A/B, alternating
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6f
mkdir -p $O
L=$GRAFT_REPO_ROOT/mujocoposelearning_amd
timeout -k 10 120 python tools/probes/gpu_hash_steps.py > $O/hash.txt 2>&1 || exit 3
HSIM_LIB=$L/libhsim_la.so timeout -k 10 120 python tools/probes/gpu_hash_steps.py >> $O/hash.txt 2>&1 || exit 4
B="python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-rollout --no-gae --train-iters 0 --no-configs --no-fp32 --no-episodes --no-tape --no-dropin"
for i in 1 2 3; do
  timeout -k 10 300 $B > $O/ab_def_$i.log 2>&1 || exit 5
  HSIM_LIB=$L/libhsim_la.so timeout -k 10 300 $B > $O/ab_la_$i.log 2>&1 || exit 6
done
