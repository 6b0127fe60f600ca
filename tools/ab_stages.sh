#!/bin/bash
# Interleaved A/B of library builds: concurrent throughput (the bench's timed loop)
# and the serialized per-stage times, per run one line in gpurun_out/$TAG/stages.txt.
#   LIBS="ros_vision_amd/ab/x.so ros_vision_amd/libat_hip.so" ROUNDS=2 TAG=ab bash tools/ab_stages.sh
set -uo pipefail
TAG=${TAG:-ab}; OUT=$(pwd)/gpurun_out/$TAG; mkdir -p $OUT
REV=$(echo $LIBS | tr ' ' '\n' | tac | tr '\n' ' ')
for r in $(seq 1 ${ROUNDS:-2}); do
  ORDER=$LIBS
  if [ $((r % 2)) = 0 ]; then ORDER=$REV; fi  # even rounds backwards: no position bias
  for lib in $ORDER; do
    AT_HIP_LIB=$lib timeout -k 10 150 python3 bench.py --steps ${STEPS:-100} --warmup 5 --no-cpu-baseline \
      --latency-frames ${LATFRAMES:-0} --host-ingest-steps 0 --c3-latency-iters 0 --node-path-calls 0 --no-kernel-timer --pool 128 \
      2>>$OUT/err.txt | python3 -c "
import json,sys; j=json.load(sys.stdin)
print('round=$r lib=$lib', j['value'], j['p50_latency_hbm_ms'], ' '.join('%s=%.4f' % kv for kv in j['stage_ms_per_batch'].items()))" >> $OUT/stages.txt || exit 1
  done
done
cat $OUT/stages.txt
