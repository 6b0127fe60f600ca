#!/bin/bash
# Throughput vs. batches in flight (detector instances) and frames per step,
# interleaved rounds on one box.  CFGS="inst batch hwq;..."  Output: gpurun_out/$TAG/r.txt
set -uo pipefail
TAG=${TAG:-inst}; OUT=$(pwd)/gpurun_out/$TAG; mkdir -p $OUT
IFS=';' read -ra LIST <<< "${CFGS:-4 128 8;6 128 8}"
for r in $(seq 1 ${ROUNDS:-2}); do
  for cfg in "${LIST[@]}"; do
    read -r inst batch hwq <<< "$cfg"
    echo -n "round=$r inst=$inst batch=$batch hwq=$hwq " >> $OUT/r.txt
    timeout -k 10 150 python3 bench.py --instances $inst --batch $batch --hw-queues $hwq --pool 128 \
      --steps $((25600 / batch)) --warmup 5 --no-cpu-baseline --latency-frames 0 --no-stage-profile --no-kernel-timer \
      2>>$OUT/err.txt | python3 -c "import json,sys; j=json.load(sys.stdin); print(j['value'], j['ms_per_step'])" >> $OUT/r.txt || exit 1
  done
done
cat $OUT/r.txt
