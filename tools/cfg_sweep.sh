#!/bin/bash
# Concurrent throughput of bench configurations (batch x instances), interleaved rounds.
#   CFGS="192x4 256x4" ROUNDS=2 TAG=sw bash tools/cfg_sweep.sh
set -uo pipefail
O=gpurun_out/${TAG:-sweep}; mkdir -p $O
LEG="--no-cpu-baseline --latency-frames 0 --host-ingest-steps 0 --c3-latency-iters 0 --node-path-calls 0 --isolated-batches 0 --no-stage-profile"
for r in $(seq 1 ${ROUNDS:-2}); do for c in ${CFGS}; do
  b=${c%x*}; i=${c#*x}
  echo -n "round=$r batch=$b instances=$i " >> $O/sweep.txt
  timeout -k 10 200 python3 bench.py --steps ${STEPS:-100} --warmup 5 --batch $b --instances $i $LEG 2>>$O/sweep.err \
    | python3 -c "import json,sys; j=json.load(sys.stdin); print(j['value'], j['ms_per_step'])" >> $O/sweep.txt || exit 1
done; done
cat $O/sweep.txt
