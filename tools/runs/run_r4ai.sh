# round 4 ai: SURVEY 8(d) protocol (T0/T1/T2 x seeds 0-2, 1000 warm-up + 10000 timed env steps, 4096
# fp64 envs) with the timed steps as hs_step_tape calls of 500 steps
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4ai
timeout -k 10 900 python -u bench.py --protocol --protocol-tape --precision fp64 > gpurun_out/r4ai/protocol_tape_fp64.log 2>&1 || exit 2
