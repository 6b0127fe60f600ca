#!/bin/bash
# bench's live dominant-kernel time vs rocprofv3's average for the same command
TAG=${TAG:-ta1}; ROOT=$(pwd); OUT=$ROOT/gpurun_out/$TAG; mkdir -p $OUT
B="$ROOT/bench.py --no-cpu-baseline --no-stage-profile --latency-frames 0 --steps 40 --warmup 3"
timeout -k 10 200 python3 $B > $OUT/plain.json 2>>$OUT/err.txt || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- python3 $B > $OUT/traced.json 2>>$OUT/err.txt || exit 1
