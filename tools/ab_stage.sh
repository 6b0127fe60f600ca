#!/bin/bash
# A/B of library variants by serialized per-stage GPU time (bench.py's stage
# profile: HIP events between the kernels of one launch sequence, 10 batches),
# less noisy than concurrent throughput.  Same box, interleaved.
#   LIBS="ros_vision_amd/ab/a.so ros_vision_amd/ab/b.so" ROUNDS=2 TAG=abs bash tools/ab_stage.sh
set -uo pipefail
TAG=${TAG:-abs}; OUT=$(pwd)/gpurun_out/$TAG; mkdir -p $OUT
for r in $(seq 1 ${ROUNDS:-2}); do
  for lib in $LIBS; do
    echo -n "round=$r lib=$(basename $lib) " >> $OUT/r.txt
    AT_HIP_LIB=$lib timeout -k 10 150 python3 bench.py --batch ${BATCH:-128} --pool 128 --steps ${STEPS:-40} --warmup 3 \
      --no-cpu-baseline --latency-frames ${LATFRAMES:-0} --no-kernel-timer 2>>$OUT/err.txt | python3 -c "
import json,sys; j=json.load(sys.stdin); st=j['stage_ms_per_batch']
print('fps %.0f sum %.4f p50hbm %s' % (j['value'], sum(st.values()), j.get('p50_latency_hbm_ms')), ' '.join('%s=%.4f' % (k[2:], v) for k, v in st.items()))" >> $OUT/r.txt || exit 1
  done
done
cat $OUT/r.txt
