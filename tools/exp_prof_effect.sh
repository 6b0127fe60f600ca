#!/bin/bash
# Why is the bench faster under rocprofv3 --kernel-trace?  Plain runs with queue /
# instance variants next to a traced run.  Output: gpurun_out/$TAG/r.txt
TAG=${TAG:-pe1}; ROOT=$(pwd); OUT=$ROOT/gpurun_out/$TAG; mkdir -p $OUT
B="$ROOT/bench.py --no-cpu-baseline --no-stage-profile --latency-frames 0 --steps 40 --warmup 3"
summ() { python3 -c "import json,sys; j=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(j['value'], j['roofline']['avg_launch_ms'])"; }
run() { echo -n "$1: " >> $OUT/r.txt; shift; timeout -k 10 120 "$@" 2>>$OUT/err.txt | summ >> $OUT/r.txt || exit 1; }
run "plain hwq8 inst4" python3 $B
run "plain hwq4 inst4" python3 $B --hw-queues 4
run "plain hwq8 inst2" python3 $B --instances 2
run "plain hwq2 inst4" python3 $B --hw-queues 2
run "plain hwq1 inst4" python3 $B --hw-queues 1
cd /tmp && export TMPDIR=/tmp
run "rocprof kt hwq8 inst4" rocprofv3 --kernel-trace -d $OUT/kt -o run -- python3 $B
cd $ROOT
run "plain hwq8 inst4 again" python3 $B
