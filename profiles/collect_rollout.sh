#!/bin/bash
# rocprofv3 evidence for the train leg's dominant kernel, the fused rollout step_kernel_queue<double,27,false,true>
# (hs_rollout): kernel trace + stats, then separate PMC passes (HBM bytes; L2 read requests from the CUs, i.e.
# the pi-net weight stream; SQ busy / wait), kernel-trace only.  Outputs under gpurun_out/prof_<tag>/;
# summarized by profiles/summarize_rollout.py <tag>.
set -uo pipefail
TAG=${1:-r6_rollout}
OUT=gpurun_out/prof_${TAG}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
BENCH="python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-rollout --no-gae --train-iters 2 --no-configs --no-fp32 --no-episodes --no-tape --no-dropin --no-precondition"
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o trace -- $BENCH > "$OUT/bench_trace.log" 2>&1 || exit 21
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/fetch" -o fetch -- $BENCH > "$OUT/bench_fetch.log" 2>&1 || exit 22
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/write" -o write -- $BENCH > "$OUT/bench_write.log" 2>&1 || exit 23
timeout -s KILL 300 rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum --kernel-trace --output-format csv -d "$OUT/tcp" -o tcp -- $BENCH > "$OUT/bench_tcp.log" 2>&1 || exit 24
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU --kernel-trace --output-format csv -d "$OUT/sq" -o sq -- $BENCH > "$OUT/bench_sq.log" 2>&1 || exit 25
echo done
