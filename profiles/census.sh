#!/bin/bash
# Dynamic instruction census of the fp64 step kernel: rocprofv3 SQ_INSTS_* passes of
# the default bench window (each pass within the 8-SQ-counter limit, kernel-trace only), then one
# stochastic PC-sampling pass (no counters) for the per-instruction picture.
# Outputs under gpurun_out/census_<tag>/ ; summarized by tools/census_report.py <tag>.
set -uo pipefail
TAG=${1:-r6}
OUT=gpurun_out/census_${TAG}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
BENCH="python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-rollout --no-gae --train-iters 0 --no-configs --no-fp32 --no-episodes --no-tape --no-dropin"
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT --kernel-trace --output-format csv -d "$OUT/v1" -o v1 -- $BENCH > "$OUT/v1.log" 2>&1 || exit 11
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_BRANCH --kernel-trace --output-format csv -d "$OUT/v2" -o v2 -- $BENCH > "$OUT/v2.log" 2>&1 || exit 12
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_IOPS SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_ANY --kernel-trace --output-format csv -d "$OUT/v3" -o v3 -- $BENCH > "$OUT/v3.log" 2>&1 || exit 13
echo counters done
