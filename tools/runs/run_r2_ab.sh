# A/B: fp64 rsqrt (v_rsq + Newton steps vs correctly rounded 1/sqrt) in the phase timing build; PGS probe
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/probes/gpu_timing.py fp64 staggered > gpurun_out/timing_a.log 2>&1 || exit 1
HSIM_TIMING_LIB=$GRAFT_REPO_ROOT/mujocoposelearning_amd/libhsim_timing_b.so timeout -k 10 200 python -u tools/probes/gpu_timing.py fp64 staggered > gpurun_out/timing_b.log 2>&1 || exit 2
timeout -k 10 400 python -u tools/probes/gpu_pgs_probe2.py > gpurun_out/pgs_probe2.log 2>&1 || exit 3
