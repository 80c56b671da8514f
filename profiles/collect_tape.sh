#!/bin/bash
# rocprofv3 evidence for the tape launch (hs_step_tape, every step's obs / reward / done written, as bench.py's
# tape leg) beside the per-step launches of the same run:
# kernel trace + stats, FETCH_SIZE / WRITE_SIZE passes and the SQ issue / stall pass (one pass each).
# Outputs under gpurun_out/prof_<tag>/ ; summarize with python profiles/summarize_tape.py <tag>.
set -euo pipefail
TAG=${1:-r4w}
OUT=gpurun_out/prof_${TAG}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
BENCH="python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-rollout --no-gae --train-iters 0 --no-configs --no-fp32 --no-episodes --no-dropin --precision fp64"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o trace -- $BENCH > "$OUT/bench_trace.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/fetch" -o fetch -- $BENCH > "$OUT/bench_fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/write" -o write -- $BENCH > "$OUT/bench_write.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d "$OUT/sq" -o sq -- $BENCH > "$OUT/bench_sq.log" 2>&1
echo done
