# Per-phase cycle split of the fp64 step kernel (diagnostic build: make -C mujocoposelearning_amd/csrc timing)
# at 4096 envs over the staggered episode mix, and at the reference's own n_envs = 8.
#   gpurun -- 'bash tools/runs/timing.sh r6g'
TAG=${1:?usage: timing.sh TAG}
cd $GRAFT_REPO_ROOT
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 200 python tools/probes/gpu_timing.py fp64 staggered > $O/timing_4096.txt 2>&1 || exit 3
timeout -k 10 200 python tools/probes/gpu_timing.py fp64 n=8 > $O/timing_8.txt 2>&1 || exit 4
