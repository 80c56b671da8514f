# round 4 ae: fused-rollout policy forward with a weight-row ring (HS_POL_RING 16) -- rollout + PPO
# GPU tests, then the rollout cost probe A/B against the previous library (HSIM_LIB=libhsim_base.so)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4ae
timeout -k 10 400 python -u -m pytest tests/test_gpu_rollout.py tests/test_gpu_ppo.py -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/r4ae/tests.log 2>&1 || exit 2
for v in base new base new; do
  if [ $v == base ]; then L="HSIM_LIB=$PWD/mujocoposelearning_amd/libhsim_base.so"; else L="HSIM_LIB=$PWD/mujocoposelearning_amd/libhsim.so"; fi
  echo "== $v" >> gpurun_out/r4ae/ab.log
  env $L timeout -k 10 200 python -u tools/probes/gpu_rollout_cost.py >> gpurun_out/r4ae/ab.log 2>&1 || exit 3
done
