#!/bin/bash
# bench value + stage times under environment variants: ENVS="A=1 B=2;C=3" (';'-separated)
TAG=${TAG:-env}; mkdir -p gpurun_out/$TAG
IFS=';' read -ra VARS <<< "$ENVS"
for v in "${VARS[@]}"; do
  echo -n "[$v] " >> gpurun_out/$TAG/r.txt
  env $v timeout -k 10 120 python bench.py --no-cpu-baseline --latency-frames 20 ${BENCH_ARGS} | python -c "import json,sys; j=json.load(sys.stdin); print(j['value'], j['p50_latency_ms'], j['stage_ms_per_batch'])" >> gpurun_out/$TAG/r.txt || exit 1
done
