#!/bin/bash
# SQ counter passes over a short bench run (one pass per counter group, no
# tracing combined with --pmc).  Output: gpurun_out/$TAG/pmc_*/
set -euo pipefail
TAG=${1:-sq}
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
ARGS="$ROOT/bench.py --no-cpu-baseline --no-stage-profile --steps 4 --warmup 1 --latency-frames 0"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --output-format csv -d "$OUT/pmc_a" -o run -- python3 $ARGS > /dev/null 2> "$OUT/pmc_a.err"
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM SQ_WAIT_INST_LDS --output-format csv -d "$OUT/pmc_b" -o run -- python3 $ARGS > /dev/null 2> "$OUT/pmc_b.err"
