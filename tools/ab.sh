#!/bin/bash
# A/B throughput of library variants in one GPU call (same box, interleaved runs).
#   LIBS="ros_vision_amd/libat_hip.so /tmp/x.so ..." CFG="4 128 8" ROUNDS=2 TAG=ab bash tools/ab.sh
set -uo pipefail
TAG=${TAG:-ab}; OUT=$(pwd)/gpurun_out/$TAG; mkdir -p $OUT
read -r inst batch hwq <<< "${CFG:-4 128 8}"
REV=$(echo $LIBS | tr ' ' '\n' | tac | tr '\n' ' ')
for r in $(seq 1 ${ROUNDS:-2}); do
  ORDER=$LIBS
  if [ "${ALT:-0}" = 1 ] && [ $((r % 2)) = 0 ]; then ORDER=$REV; fi  # even rounds backwards: no position bias
  for lib in $ORDER; do
    echo -n "round=$r lib=$lib " >> $OUT/r.txt
    AT_HIP_LIB=$lib timeout -k 10 150 python3 bench.py --instances $inst --batch $batch --hw-queues $hwq --pool 128 \
      --steps ${STEPS:-100} --warmup 5 --no-cpu-baseline --latency-frames ${LATFRAMES:-0} --host-ingest-steps 0 --c3-latency-iters 0 --no-stage-profile --no-kernel-timer \
      2>>$OUT/err.txt | python3 -c "import json,sys; j=json.load(sys.stdin); print(j['value'], j['ms_per_step'], j['p50_latency_hbm_ms'])" >> $OUT/r.txt || exit 1
  done
done
cat $OUT/r.txt
