# SURVEY 8(d) protocol: per tape T0/T1/T2 x base seed {0,1,2}: reset, 1000 warm-up + 10000 timed env steps
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r2i
timeout -k 10 500 python -u bench.py --protocol --precision fp64 > gpurun_out/r2i/protocol_fp64.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --protocol --precision fp32 > gpurun_out/r2i/protocol_fp32.log 2>&1 || exit 2
