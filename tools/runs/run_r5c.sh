# round 5 c: SURVEY 8(d) protocol (per-step launches and 500-step tape calls, fp64), the 1000-substep
# parity report, and the drop-in leg again (longer warm-up)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5c
timeout -k 10 400 python -u bench.py --protocol --precision fp64 > gpurun_out/r5c/protocol_fp64.log 2>&1 || exit 2
timeout -k 10 400 python -u bench.py --protocol --protocol-tape --precision fp64 > gpurun_out/r5c/protocol_tape_fp64.log 2>&1 || exit 3
timeout -k 10 400 python -u tools/probes/parity_report.py > gpurun_out/r5c/parity_report.md 2> gpurun_out/r5c/parity_report.err || exit 4
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-rollout --no-gae --train-iters 0 --no-configs --no-fp32 --no-episodes --no-tape > gpurun_out/r5c/dropin.log 2>&1 || exit 5
