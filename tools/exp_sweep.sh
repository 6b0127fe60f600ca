#!/bin/bash
# throughput vs batch and batches in flight.  CFGS="inst batch;..."
TAG=${TAG:-sw}; ROOT=$(pwd); OUT=$ROOT/gpurun_out/$TAG; mkdir -p $OUT
IFS=';' read -ra LIST <<< "${CFGS:-4 32}"
timeout -k 10 200 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || exit 1
for cfg in "${LIST[@]}"; do
  read -r inst batch <<< "$cfg"
  echo -n "inst=$inst batch=$batch " >> $OUT/r.txt
  timeout -k 10 150 python3 bench.py --instances $inst --batch $batch --pool 128 --steps 30 --warmup 3 --no-cpu-baseline --latency-frames 0 --no-stage-profile 2>>$OUT/err.txt | python3 -c "import json,sys; j=json.load(sys.stdin); print(j['value'], j['ms_per_step'], j['roofline']['avg_launch_ms'])" >> $OUT/r.txt || exit 1
done
