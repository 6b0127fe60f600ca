#!/bin/bash
# Throughput vs detector instances (batches in flight), frames per step and HW
# queues.  CFGS="inst batch hwq;..."   Output: gpurun_out/$TAG/r.txt
set -uo pipefail
TAG=${TAG:-sw}; ROOT=$(pwd); OUT=$ROOT/gpurun_out/$TAG; mkdir -p $OUT
IFS=';' read -ra LIST <<< "${CFGS:-4 32 8}"
for cfg in "${LIST[@]}"; do
  read -r inst batch hwq <<< "$cfg"
  echo -n "inst=$inst batch=$batch hwq=$hwq " >> $OUT/r.txt
  timeout -k 10 150 python3 bench.py --instances $inst --batch $batch --hw-queues $hwq --pool 128 --steps ${STEPS:-40} --warmup 5 \
    --no-cpu-baseline --latency-frames 0 --host-ingest-steps 0 --c3-latency-iters 0 --no-stage-profile --no-kernel-timer 2>>$OUT/err.txt \
    | python3 -c "import json,sys; j=json.load(sys.stdin); print(j['value'], j['ms_per_step'], j.get('detections_per_frame'), j.get('host_us_per_step'))" >> $OUT/r.txt || exit 1
done
cat $OUT/r.txt
