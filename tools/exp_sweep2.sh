#!/bin/bash
# throughput vs (hw queues, instances, batch).  CFGS="hwq inst batch;..."
TAG=${TAG:-sw}; ROOT=$(pwd); OUT=$ROOT/gpurun_out/$TAG; mkdir -p $OUT
IFS=';' read -ra LIST <<< "${CFGS:-8 4 32}"
for cfg in "${LIST[@]}"; do
  read -r hwq inst batch <<< "$cfg"
  echo -n "hwq=$hwq inst=$inst batch=$batch " >> $OUT/r.txt
  timeout -k 10 150 python3 bench.py --hw-queues $hwq --instances $inst --batch $batch --steps 40 --warmup 4 --no-cpu-baseline --latency-frames 0 --no-stage-profile 2>>$OUT/err.txt | python3 -c "import json,sys; j=json.load(sys.stdin); print(j['value'], j['ms_per_step'])" >> $OUT/r.txt || exit 1
done
