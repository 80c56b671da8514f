# round 4 u: fused-rollout policy forward unroll A/B (HSIM_LIB variants)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4u
for v in base u1 u4 u8 base; do
  if [ $v == base ]; then L=""; else L="HSIM_LIB=$PWD/mujocoposelearning_amd/libhsim_$v.so"; fi
  echo "== $v" >> gpurun_out/r4u/ab.log
  env $L timeout -k 10 200 python -u tools/probes/gpu_rollout_cost.py >> gpurun_out/r4u/ab.log 2>&1 || exit 2
done
