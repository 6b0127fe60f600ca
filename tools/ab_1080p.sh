#!/bin/bash
# 1920x1080 throughput of library builds (LIBS) at batch sizes (BATCHES), interleaved
O=gpurun_out/${TAG:-ab1080}; mkdir -p $O
for r in 1 2; do for lib in ${LIBS:-ros_vision_amd/ab/libat_prev.so ros_vision_amd/libat_hip.so}; do for b in ${BATCHES:-128 192}; do
  echo -n "r=$r lib=$lib batch=$b " >> $O/r.txt
  AT_HIP_LIB=$lib timeout -k 10 200 python3 bench.py --width 1920 --height 1080 --tags 24 --batch $b --steps 40 --no-cpu-baseline --latency-frames 0 --host-ingest-steps 0 --c3-latency-iters 0 --node-path-calls 0 --no-kernel-timer 2>>$O/err.txt | python3 -c "import json,sys; j=json.load(sys.stdin); print(j['value'], j['detections_per_frame'], ' '.join('%s=%.4f' % kv for kv in j['stage_ms_per_batch'].items()))" >> $O/r.txt || exit 1
done; done; done
