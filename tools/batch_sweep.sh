#!/bin/bash
# Throughput vs. frames per step (bench.py --batch), plus one kernel-trace
# timeline of the steady state.  Output: gpurun_out/$TAG/
set -euo pipefail
TAG=${1:-sweep}
OUT=$(pwd)/gpurun_out/$TAG
mkdir -p "$OUT"
for b in ${BATCHES:-16 32 64 128}; do
  echo -n "batch=$b " >> "$OUT/sweep.txt"
  timeout -k 10 150 python bench.py --batch $b --pool 128 --steps 20 --warmup 3 --no-cpu-baseline --latency-frames 0 --no-stage-profile \
    | python -c "import json,sys; j=json.load(sys.stdin); print(j['value'], j['ms_per_step'])" >> "$OUT/sweep.txt"
done
export TMPDIR=/tmp
ROOT=$(pwd)
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$OUT/timeline" -o run -- python3 $ROOT/bench.py --no-cpu-baseline --no-stage-profile --steps 10 --warmup 3 --latency-frames 0 > "$OUT/timeline_bench.json" 2> "$OUT/timeline.err"
