# per-phase timing of the current kernel; A/B: cubic fp64 reciprocal (r3), straight-line contact aggregates (ag)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/probes/gpu_timing.py fp64 staggered > gpurun_out/r3ai_timing_fp64.txt 2>&1 || exit 1
bash profiles/ab.sh r3ai mujocoposelearning_amd/libhsim.so mujocoposelearning_amd/libhsim_r3.so mujocoposelearning_amd/libhsim_ag.so || exit 2
