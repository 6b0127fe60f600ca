# round-5 GPU call; steps selected by environment variables:
#   GPU_TESTS=1  pytest -m gpu (a failing test is recorded, a crash ends the call)
#   BENCH=1      the default bench line -> bench.json
#   LIBS="a.so b.so"     interleaved concurrent A/B (tools/ab_stages.sh)
#   PMCLIBS="a.so b.so"  FETCH / WRITE bytes per kernel of each library (tools/pmc_ab.sh)
#   LDSLIBS="a.so b.so"  LDS instructions, bank conflicts, wave-cycles per kernel of each library
#   ISO=1        bench.py --isolated-only under rocprofv3 --kernel-trace --stats, roofline_check
#   SQX=1        per-class VALU counter passes + tools/valu_rates (issue costs)
# usage: TAG=r05b GPU_TESTS=1 ... bash tools/r05_call.sh
set -o pipefail
TAG=${TAG:-r05}; O=gpurun_out/$TAG; mkdir -p $O
R=$(pwd)
export TMPDIR=/tmp
if [ -n "${LIST:-}" ]; then timeout -k 10 60 rocprofv3 -L > $O/counters.txt 2>&1 || true; fi
if [ -n "${GPU_TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1
  rc=$?; echo "tests rc=$rc" >> $O/rc.txt
  case $rc in 0|1) ;; *) exit $rc;; esac
fi
if [ -n "${BENCH:-}" ]; then
  timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || exit 1
fi
if [ -n "${TIMER_AB:-}" ]; then  # the timed region with and without the live kernel timer, interleaved
  LEG="--no-cpu-baseline --latency-frames 0 --host-ingest-steps 0 --c3-latency-iters 0 --node-path-calls 0 --no-stage-profile --isolated-batches 0"
  for r in 1 2 3; do for t in "" "--no-kernel-timer"; do
    echo -n "round=$r timer=${t:-on} " >> $O/timer_ab.txt
    timeout -k 10 200 python3 bench.py $LEG $t 2>>$O/timer_ab.err | python3 -c "import json,sys; j=json.load(sys.stdin); print(j['value'], j['ms_per_step'])" >> $O/timer_ab.txt || exit 1
  done; done
fi
if [ -n "${LIBS:-}" ]; then TAG=$TAG bash tools/ab_stages.sh > /dev/null || exit 1; fi
if [ -n "${PMCLIBS:-}" ]; then LIBS="$PMCLIBS" TAG=$TAG/pmc bash tools/pmc_ab.sh > $O/pmc_ab.txt 2> $O/pmc_ab.err || exit 1; fi
if [ -n "${LDSLIBS:-}" ]; then  # LDS instructions / bank conflicts / wave-cycles per kernel of each library
  SHORTL="$R/bench.py --no-cpu-baseline --no-stage-profile --batch 192 --steps 4 --warmup 1 --latency-frames 0 --host-ingest-steps 0 --c3-latency-iters 0 --node-path-calls 0 --isolated-batches 0"
  for lib in $LDSLIBS; do
    n=$(basename $lib .so)
    (cd /tmp && AT_HIP_LIB=$R/$lib timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_WAIT_ANY \
       --output-format csv -d $R/$O/lds_$n -o run -- python3 $SHORTL > /dev/null 2> $R/$O/lds_$n.err) || exit 1
    python3 tools/pmc_agg.py $O/lds_$n/run_counter_collection.csv > $O/lds_$n.txt
  done
fi
if [ -n "${ISO:-}" ]; then
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/trace_iso -o run -- \
     python3 $R/bench.py --isolated-only > $R/$O/iso_traced.json 2> $R/$O/iso_traced.err) || exit 1
  if [ -s $O/bench.json ]; then
    python3 tools/roofline_check.py $O/trace_iso/run_kernel_stats.csv $O/bench.json $O/iso_traced.json > $O/roofline_check.json
  fi
  python3 tools/roofline_check.py $O/trace_iso/run_kernel_stats.csv $O/iso_traced.json > $O/roofline_check_traced.json
fi
if [ -n "${SQX:-}" ]; then
  SHORT="$R/bench.py --no-cpu-baseline --no-stage-profile --batch 192 --steps 4 --warmup 1 --latency-frames 0 --host-ingest-steps 0 --c3-latency-iters 0 --node-path-calls 0 --isolated-batches 0"
  (cd /tmp && timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 \
     SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT GRBM_GUI_ACTIVE \
     --output-format csv -d $R/$O/pmc_sq_c -o run -- python3 $SHORT > /dev/null 2> $R/$O/pmc_sq_c.err) || exit 1
  (cd /tmp && timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 \
     SQ_INSTS_VALU_INT32 SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE \
     --output-format csv -d $R/$O/pmc_sq_d -o run -- python3 $SHORT > /dev/null 2> $R/$O/pmc_sq_d.err) || exit 1
  (cd /tmp && timeout -s KILL 240 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM \
     SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU GRBM_GUI_ACTIVE \
     --output-format csv -d $R/$O/pmc_sq_e -o run -- python3 $SHORT > /dev/null 2> $R/$O/pmc_sq_e.err) || exit 1
  python3 tools/pmc_agg.py $O/pmc_sq_c/run_counter_collection.csv $O/pmc_sq_d/run_counter_collection.csv \
     $O/pmc_sq_e/run_counter_collection.csv > $O/sq_counters_agg.txt
  timeout -k 10 120 tools/valu_rates > $O/valu_rates.jsonl || exit 1
  (cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/trace_sq -o run -- python3 $SHORT > /dev/null 2> $R/$O/trace_sq.err) || exit 1
fi
echo ok >> $O/rc.txt
