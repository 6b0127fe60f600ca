#!/bin/bash
# Interleaved A/B of environment settings (knobs read by at_create) on one library
# (the experiment build, make -C ros_vision_amd/csrc exp: the product library ignores them):
# concurrent throughput of the bench loop and serialized stage times, one line per run.
#   ENVS="AT_X=1 AT_X=2" ROUNDS=4 TAG=ab bash tools/ab_envs.sh
set -uo pipefail
TAG=${TAG:-ab}; OUT=$(pwd)/gpurun_out/$TAG; mkdir -p $OUT
REV=$(echo $ENVS | tr ' ' '\n' | tac | tr '\n' ' ')
for r in $(seq 1 ${ROUNDS:-2}); do
  ORDER=$ENVS
  if [ $((r % 2)) = 0 ]; then ORDER=$REV; fi
  for ev in $ORDER; do
    env AT_HIP_LIB=${AT_HIP_LIB:-ros_vision_amd/ab/libat_hip_exp.so} $ev timeout -k 10 150 python3 bench.py --steps ${STEPS:-100} --warmup 5 --no-cpu-baseline \
      --latency-frames 0 --host-ingest-steps 0 --c3-latency-iters 0 --node-path-calls 0 --no-kernel-timer --pool 128 \
      2>>$OUT/err.txt | python3 -c "
import json,sys; j=json.load(sys.stdin)
print('round=$r lib=$ev', j['value'], j['p50_latency_hbm_ms'], ' '.join('%s=%.4f' % kv for kv in j['stage_ms_per_batch'].items()))" >> $OUT/stages.txt || exit 1
  done
done
