#!/bin/bash
# round-6 GPU call; steps selected by environment variables (outputs: gpurun_out/$TAG/):
#   GPU_TESTS=1        pytest -m gpu (a failing test is recorded, a crash ends the call)
#   TESTS="files..."   only these test files (-m gpu)
#   ABL=1              stage-cut ablation at the bench configuration (4 x 192, 720p):
#                      throughput with the launch sequence cut after each stage
#                      (AT_DIAG_PIPE_STOP, experiment build) -> ablation.txt
#   ABL1080=1          the same at 1920x1080
#   P1080=1            1080p profile: bench line with stage profile + isolated kernels,
#                      FETCH / WRITE passes (pmc_traffic_1080p.json)
#   BENCH=1            the default bench line -> bench.json
#   BSTOPS="0 2 3 4 7 8"  blob kernels cut after a phase (experiment build): serialized stage ms
#   LATLIBS="a b"      B = 1 latency (p50 / p99 from HBM) of each library, three interleaved rounds
#   LIBS="a.so b.so"   interleaved concurrent A/B at 720p (tools/ab_stages.sh)
#   LIBS1080="a b"     the same at 1080p
#   ENVS="AT_X=1 AT_X=2"  interleaved A/B of experiment-build knobs (tools/ab_envs.sh)
#   PMCLIBS="a b"      FETCH / WRITE bytes per kernel of each library (tools/pmc_ab.sh)
#   ISO=1              bench.py --isolated-only under rocprofv3 --kernel-trace --stats
set -o pipefail
TAG=${TAG:-r06}; O=gpurun_out/$TAG; mkdir -p $O
R=$(pwd)
export TMPDIR=/tmp
EXP=${EXP:-ros_vision_amd/ab/libat_hip_exp.so}
fatal() { case $1 in 0|1) return 0;; *) echo "fatal rc=$1" >> $O/fatal.txt; exit $1;; esac; }
if [ -n "${GPU_TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest ${TESTS:-tests} -m gpu -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1
  rc=$?; echo "tests rc=$rc" >> $O/rc.txt; fatal $rc
fi
if [ -n "${BENCH:-}" ]; then
  timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || exit 1
fi
ablate() {  # $1 = output file, rest = bench geometry options
  out=$1; shift
  for ps in ${PSTOPS:-0 1 2 3 5 6 7 8 9 10 11 12}; do
    echo -n "pipe_stop=$ps " >> $out
    AT_HIP_LIB=$EXP AT_DIAG_PIPE_STOP=$ps timeout -k 10 200 python3 bench.py "$@" --steps ${STEPS:-100} --warmup 5 --no-cpu-baseline \
      --latency-frames 0 --host-ingest-steps 0 --c3-latency-iters 0 --node-path-calls 0 --no-stage-profile --no-kernel-timer \
      2>>$O/abl_err.txt | python3 -c "import json,sys; j=json.load(sys.stdin); print(j['value'], j['ms_per_step'], j['detections_per_frame'])" >> $out || exit 1
  done
}
if [ -n "${ABL:-}" ]; then ablate $O/ablation_720p.txt; fi
if [ -n "${ABL1080:-}" ]; then ablate $O/ablation_1080p.txt --width 1920 --height 1080 --tags 24; fi
if [ -n "${P1080:-}" ]; then
  G="--width 1920 --height 1080 --tags 24"
  timeout -k 10 400 python bench.py $G --steps 100 --no-cpu-baseline --host-ingest-steps 0 --c3-latency-iters 0 --node-path-calls 0 \
    --latency-frames 300 > $O/bench_1080p.json 2> $O/bench_1080p.err || exit 1
  SHORT="$R/bench.py $G --no-cpu-baseline --no-stage-profile --steps 4 --warmup 1 --latency-frames 0 --host-ingest-steps 0 --c3-latency-iters 0 --node-path-calls 0 --isolated-batches 0"
  (cd /tmp && timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/$O/pmc1080_fetch -o run -- python3 $SHORT > /dev/null 2> $R/$O/pmc1080_fetch.err) || exit 1
  (cd /tmp && timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/$O/pmc1080_write -o run -- python3 $SHORT > /dev/null 2> $R/$O/pmc1080_write.err) || exit 1
  python3 tools/pmc_traffic.py $O/pmc1080_fetch/run_counter_collection.csv $O/pmc1080_write/run_counter_collection.csv 192 1920 1080 $O/pmc_traffic_1080p.json > /dev/null || exit 1
fi
if [ -n "${BSTOPS:-}" ]; then  # blob kernels cut after phase N (AT_DIAG_BLOB_STOP): serialized stage times
  for r in 1 2; do for st in $BSTOPS; do
    echo -n "round=$r blob_stop=$st " >> $O/blob_stops.txt
    AT_HIP_LIB=$EXP AT_DIAG_BLOB_STOP=$st timeout -k 10 200 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --latency-frames 0 \
      --host-ingest-steps 0 --c3-latency-iters 0 --node-path-calls 0 --no-kernel-timer 2>>$O/err.txt | python3 -c "
import json,sys; j=json.load(sys.stdin); s=j['stage_ms_per_batch']; print(j['value'], 'k_blob_small=%.4f k_blob=%.4f k_decode=%.4f' % (s['k_blob_small'], s['k_blob'], s['k_decode']))" >> $O/blob_stops.txt || exit 1
  done; done
fi
if [ -n "${LATLIBS:-}" ]; then  # B = 1 latency of each library, interleaved rounds
  for r in 1 2 3; do for lib in $LATLIBS; do
    echo -n "round=$r lib=$lib " >> $O/lat.txt
    AT_HIP_LIB=$lib timeout -k 10 200 python3 bench.py --steps 3 --warmup 2 --latency-frames ${LATN:-2000} --no-cpu-baseline --no-stage-profile \
      --no-kernel-timer --host-ingest-steps 0 --c3-latency-iters 0 --node-path-calls 0 --isolated-batches 0 2>>$O/err.txt | python3 -c "
import json,sys; j=json.load(sys.stdin); print('p50 %.4f p99 %.4f' % (j['p50_latency_hbm_ms'], j['p99_latency_hbm_ms']))" >> $O/lat.txt || exit 1
  done; done
fi
if [ -n "${LIBS:-}" ]; then TAG=$TAG bash tools/ab_stages.sh > /dev/null || exit 1; fi
if [ -n "${ENVS:-}" ]; then TAG=$TAG bash tools/ab_envs.sh > /dev/null || exit 1; fi
if [ -n "${LIBS1080:-}" ]; then
  for r in 1 2; do for lib in $LIBS1080; do
    echo -n "round=$r lib=$lib " >> $O/ab1080.txt
    AT_HIP_LIB=$lib timeout -k 10 200 python bench.py --width 1920 --height 1080 --tags 24 --steps ${STEPS1080:-60} --no-cpu-baseline --latency-frames 0 \
      --host-ingest-steps 0 --c3-latency-iters 0 --node-path-calls 0 --no-kernel-timer --isolated-batches 0 2>>$O/err.txt | python3 -c "
import json,sys; j=json.load(sys.stdin); print(j['value'], j['detections_per_frame'], ' '.join('%s=%.4f' % kv for kv in j['stage_ms_per_batch'].items()))" >> $O/ab1080.txt || exit 1
  done; done
fi
if [ -n "${PMCLIBS:-}" ]; then LIBS="$PMCLIBS" TAG=$TAG/pmc bash tools/pmc_ab.sh > $O/pmc_ab.txt 2> $O/pmc_ab.err || exit 1; fi
if [ -n "${ISO:-}" ]; then
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/trace_iso -o run -- \
     python3 $R/bench.py --isolated-only > $R/$O/iso_traced.json 2> $R/$O/iso_traced.err) || exit 1
  python3 tools/roofline_check.py $O/trace_iso/run_kernel_stats.csv $O/iso_traced.json > $O/roofline_check_traced.json
fi
echo ok >> $O/rc.txt
