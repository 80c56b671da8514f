# round 4 x: tape profile with per-step outputs written (bench's tape leg now does), and the SURVEY 8(d)
# protocol on the round-4 kernel
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4x
bash profiles/collect_tape.sh r4x > gpurun_out/collect_r4x.log 2>&1 || exit 7
timeout -k 10 400 python -u bench.py --protocol --precision fp64 > gpurun_out/r4x/protocol_fp64.log 2>&1 || exit 8
