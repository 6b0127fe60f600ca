#!/bin/bash
# k_pre + k_thr_ccl only (AT_DIAG_PIPE_STOP=2, experiment builds): concurrent cost of k_thr_ccl variants
#   LIBS="libat_a.so libat_b.so" (under ros_vision_amd/ab/) [PS=2] bash tools/ps2_ab.sh
O=gpurun_out/ps2; mkdir -p $O
for r in 1 2; do for lib in $LIBS; do
  echo -n "r=$r $lib " >> $O/r.txt
  AT_HIP_LIB=ros_vision_amd/ab/$lib AT_DIAG_PIPE_STOP=${PS:-2} timeout -k 10 120 python3 bench.py --steps 100 --warmup 5 --no-cpu-baseline \
    --latency-frames 0 --host-ingest-steps 0 --c3-latency-iters 0 --no-kernel-timer 2>>$O/err.txt \
    | python3 -c "import json,sys; j=json.load(sys.stdin); print(j['value'], j['ms_per_step'], j['stage_ms_per_batch'].get('k_thr_ccl'))" >> $O/r.txt || exit 1
done; done
