#!/bin/bash
# Throughput under environment variants, interleaved: ENVS="A=1;B=2;..." (an empty entry = baseline)
set -uo pipefail
TAG=${TAG:-env}; OUT=$(pwd)/gpurun_out/$TAG; mkdir -p $OUT
IFS=';' read -ra LIST <<< "${ENVS:-}"
for r in $(seq 1 ${ROUNDS:-3}); do
  for e in "${LIST[@]}"; do
    echo -n "round=$r env=[$e] " >> $OUT/r.txt
    env $e timeout -k 10 150 python3 bench.py --pool 128 --steps ${STEPS:-100} --warmup 5 --no-cpu-baseline \
      --latency-frames 0 --no-stage-profile --no-kernel-timer 2>>$OUT/err.txt \
      | python3 -c "import json,sys; j=json.load(sys.stdin); print(j['value'], j['ms_per_step'], j.get('host_us_per_step'))" >> $OUT/r.txt || exit 1
  done
done
cat $OUT/r.txt
