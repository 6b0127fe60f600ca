#!/bin/bash
# Throughput with parts of the pipeline cut off (AT_DIAG_BLOB_STOP; diagnostics only):
# the marginal cost of the later stages at the bench configuration.  The knobs exist
# only in the experiment build (make -C ros_vision_amd/csrc exp).
set -uo pipefail
TAG=${TAG:-abl}; OUT=$(pwd)/gpurun_out/$TAG; mkdir -p $OUT
for stop in ${STOPS:-0 6 5 8 4 2}; do
  echo -n "stop=$stop " >> $OUT/r.txt
  AT_HIP_LIB=${AT_HIP_LIB:-ros_vision_amd/ab/libat_hip_exp.so} AT_DIAG_BLOB_STOP=$stop timeout -k 10 150 python3 bench.py --pool 128 --steps ${STEPS:-100} --warmup 5 --no-cpu-baseline \
    --latency-frames 0 --no-stage-profile --no-kernel-timer 2>>$OUT/err.txt \
    | python3 -c "import json,sys; j=json.load(sys.stdin); print(j['value'], j['ms_per_step'], j['detections_per_frame'])" >> $OUT/r.txt || exit 1
done
cat $OUT/r.txt
for ps in ${PSTOPS:-}; do
  echo -n "pipe_stop=$ps " >> $OUT/r.txt
  AT_HIP_LIB=${AT_HIP_LIB:-ros_vision_amd/ab/libat_hip_exp.so} AT_DIAG_PIPE_STOP=$ps timeout -k 10 150 python3 bench.py --pool 128 --steps ${STEPS:-100} --warmup 5 --no-cpu-baseline \
    --latency-frames 0 --no-stage-profile --no-kernel-timer 2>>$OUT/err.txt \
    | python3 -c "import json,sys; j=json.load(sys.stdin); print(j['value'], j['ms_per_step'])" >> $OUT/r.txt || exit 1
done
cat $OUT/r.txt
