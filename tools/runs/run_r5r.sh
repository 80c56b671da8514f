# round 5 r: closing evidence on the final build: SURVEY 8(d) protocol (per-step launches and
# 500-step tape calls, fp64) and two more default bench lines (run-to-run spread)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5r
timeout -k 10 400 python -u bench.py --protocol --precision fp64 > gpurun_out/r5r/protocol_fp64.log 2>&1 || exit 2
timeout -k 10 400 python -u bench.py --protocol --protocol-tape --precision fp64 > gpurun_out/r5r/protocol_tape_fp64.log 2>&1 || exit 3
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/r5r/bench_a.log 2>&1 || exit 4
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/r5r/bench_b.log 2>&1 || exit 5
