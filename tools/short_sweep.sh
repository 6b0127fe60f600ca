#!/bin/bash
# bench.py value at the driver's short timed windows (K steps) for several
# (instances, batch) configurations, interleaved.  CFGS="inst batch;..." KS="20 40"
set -uo pipefail
TAG=${TAG:-short}; OUT=$(pwd)/gpurun_out/$TAG; mkdir -p $OUT
IFS=';' read -ra LIST <<< "${CFGS:-4 128;6 64}"
for r in $(seq 1 ${ROUNDS:-2}); do
  for k in ${KS:-20 40}; do
    for cfg in "${LIST[@]}"; do
      read -r inst batch <<< "$cfg"
      echo -n "round=$r K=$k inst=$inst batch=$batch " >> $OUT/r.txt
      timeout -k 10 150 python3 bench.py --instances $inst --batch $batch --pool ${POOL:-64} --hw-queues ${HWQ:-8} --steps $k --warmup 5 --no-cpu-baseline \
        --latency-frames 0 --no-stage-profile --timed-kernel k_blob_small 2>>$OUT/err.txt \
        | python3 -c "import json,sys; j=json.load(sys.stdin); print(j['value'], j['ms_per_step'])" >> $OUT/r.txt || exit 1
    done
  done
done
cat $OUT/r.txt
