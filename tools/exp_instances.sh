#!/bin/bash
# throughput vs. batches in flight (detector instances), blob fork on/off, HW queues, batch
# CFGS="hwq inst nofork batch;..."
TAG=${TAG:-e2}; mkdir -p gpurun_out/$TAG
IFS=';' read -ra LIST <<< "${CFGS:-4 2 0 32}"
for cfg in "${LIST[@]}"; do
  read -r hwq inst nofork batch <<< "$cfg"
  echo -n "hwq=$hwq inst=$inst nofork=$nofork batch=$batch " >> gpurun_out/$TAG/r.txt
  GPU_MAX_HW_QUEUES=$hwq AT_NO_FORK=$nofork timeout -k 10 100 python bench.py --instances $inst --batch $batch --pool 128 --steps 30 --warmup 3 --no-cpu-baseline --latency-frames 0 --no-stage-profile | python -c "import json,sys; j=json.load(sys.stdin); print(j['value'], j['ms_per_step'])" >> gpurun_out/$TAG/r.txt || exit 1
done
