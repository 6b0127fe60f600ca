#!/bin/bash
# throughput vs. batches in flight (detector instances), blob fork on/off, HW queues
mkdir -p gpurun_out/${TAG:-e2}
for cfg in ${CFGS:-"8 4 0" "8 4 1" "8 6 1" "8 3 0" "16 8 0" "8 8 1"}; do set -- $cfg
  echo -n "hwq=$1 inst=$2 nofork=$3 " >> gpurun_out/${TAG:-e2}/r.txt
  GPU_MAX_HW_QUEUES=$1 AT_NO_FORK=$3 timeout -k 10 100 python bench.py --instances $2 --steps 30 --warmup 3 --no-cpu-baseline --latency-frames 0 --no-stage-profile | python -c "import json,sys; j=json.load(sys.stdin); print(j['value'], j['ms_per_step'])" >> gpurun_out/${TAG:-e2}/r.txt || exit 1
done
