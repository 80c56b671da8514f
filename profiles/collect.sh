#!/bin/bash
# Collect rocprofv3 evidence for the step kernel on the GPU box (run from the repo root).
#   1) kernel trace + stats of the bench command (average kernel duration)
#   2) separate PMC passes for FETCH_SIZE and WRITE_SIZE (HBM bytes), kernel-trace only
#   3) SQ issue / stall counters (two passes within the per-block counter limits)
# Outputs under gpurun_out/prof_<tag>/ ; summarize with profiles/summarize.py <tag> <precision>.
set -euo pipefail
TAG=${1:-r2a}
PREC=${2:-fp64}
OUT=gpurun_out/prof_${TAG}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
BENCH="python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-rollout --no-gae --train-iters 0 --no-configs --no-fp32 --no-episodes --no-tape --no-dropin --precision $PREC"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o trace -- $BENCH > "$OUT/bench_trace.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/fetch" -o fetch -- $BENCH > "$OUT/bench_fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/write" -o write -- $BENCH > "$OUT/bench_write.log" 2>&1
# issue/stall picture of the (latency-bound) step kernel: SQ counters count quad-cycles
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d "$OUT/sq" -o sq -- $BENCH > "$OUT/bench_sq.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INST_CYCLES_SALU --kernel-trace --output-format csv -d "$OUT/sq2" -o sq2 -- $BENCH > "$OUT/bench_sq2.log" 2>&1
echo done
