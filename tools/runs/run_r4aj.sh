# round 4 aj: rocprofv3 kernel trace of bench.py's rollout + train legs (fused rollout kernel
# step_kernel_queue<double,27,false,true>, policy / update kernels), fp64, 4096 envs
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4aj
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4aj/trace -o trace -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-configs --no-fp32 --no-episodes --no-tape --no-gae --train-iters 3 > gpurun_out/r4aj/bench.log 2>&1 || exit 2
