# round 6 i: headline-window A/B -- default vs round 5's butterfly reward sums (HS_REWARD_HSUM) and two
# machine-scheduler flags on the fp64 engine (amdgpu-use-amdgpu-trackers, no unclustered high-RP reschedule)
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6i
mkdir -p $O
L=$GRAFT_REPO_ROOT/mujocoposelearning_amd
B="python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-rollout --no-gae --train-iters 0 --no-configs --no-fp32 --no-episodes --no-tape --no-dropin"
for i in 1 2; do
  timeout -k 10 300 $B > $O/ab_def_$i.log 2>&1 || exit 3
  HSIM_LIB=$L/libhsim_hsum.so timeout -k 10 300 $B > $O/ab_hsum_$i.log 2>&1 || exit 4
  HSIM_LIB=$L/libhsim_trk.so timeout -k 10 300 $B > $O/ab_trk_$i.log 2>&1 || exit 5
  HSIM_LIB=$L/libhsim_nour.so timeout -k 10 300 $B > $O/ab_nour_$i.log 2>&1 || exit 6
done
