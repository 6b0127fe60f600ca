#!/bin/bash
# Isolating the rocprofv3 speed-up: kernel timer off (graph replay), runtime-only
# trace, HSA/HIP knobs.  Output: gpurun_out/$TAG/r.txt
TAG=${TAG:-pe2}; ROOT=$(pwd); OUT=$ROOT/gpurun_out/$TAG; mkdir -p $OUT
B="$ROOT/bench.py --no-cpu-baseline --no-stage-profile --latency-frames 0 --steps 40 --warmup 3"
summ() { python3 -c "import json,sys; j=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(j['value'], j['roofline']['avg_launch_ms'])"; }
run() { echo -n "$1: " >> $OUT/r.txt; shift; timeout -k 10 120 "$@" 2>>$OUT/err.txt | summ >> $OUT/r.txt || exit 1; }
run "plain" python3 $B
run "plain no-ktimer (graph)" python3 $B --no-kernel-timer
HSA_ENABLE_INTERRUPT=0 run "HSA_ENABLE_INTERRUPT=0" python3 $B
HIP_FORCE_DEV_KERNARG=1 run "HIP_FORCE_DEV_KERNARG=1" python3 $B
run "hwq16 inst4" python3 $B --hw-queues 16
run "hwq8 inst8" python3 $B --instances 8
cd /tmp && export TMPDIR=/tmp
run "rocprof hip-runtime-trace" rocprofv3 --hip-runtime-trace -d $OUT/rt -o run -- python3 $B
run "rocprof kernel-trace no-ktimer" rocprofv3 --kernel-trace -d $OUT/kt -o run -- python3 $B --no-kernel-timer
run "rocprof memory-copy-trace" rocprofv3 --memory-copy-trace -d $OUT/mc -o run -- python3 $B
