#!/bin/bash
# One GPU call collecting this round's profiles (MI355X_MICROARCH.md HBM/rocprofv3):
#   1. rocprofv3 --kernel-trace --stats of the default bench (timed-region config)
#   2. FETCH_SIZE and WRITE_SIZE, each in its own --pmc pass (never with traces)
#   3. two SQ counter passes (8 SQ counters each)
#   4. FETCH_SIZE / WRITE_SIZE passes over tools/pmc_calib (known byte counts per
#      access width, for the gfx950 correction)
#   5. the plain bench line
# Output: gpurun_out/$TAG/...   usage: bash tools/profile_round.sh TAG [BATCH]
set -euo pipefail
TAG=${1:-prof}
BATCH=${2:-192}
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
# every profiled run is the timed loop alone (no host-ingest / C3 / latency legs), so
# the per-frame PMC figures and the rocprof averages describe the bench's timed launches
ONLY="--latency-frames 0 --host-ingest-steps 0 --c3-latency-iters 0"
SHORT="$ROOT/bench.py --no-cpu-baseline --no-stage-profile --batch $BATCH --steps 4 --warmup 1 $ONLY"
cd /tmp
# the traced run times the kernel the bench line names (its stage profile's dominant one),
# so that kernel's rocprof average and the line's live timer describe the same launches
if [ -z "${TIMED:-}" ]; then
  timeout -k 10 200 python3 $ROOT/bench.py --no-cpu-baseline --batch $BATCH --steps 4 --warmup 1 $ONLY \
    > "$OUT/dominant_probe.json" 2> "$OUT/dominant_probe.err"
  TIMED=$(python3 -c "import json,sys; print(json.load(open(sys.argv[1]))['dominant_kernel'])" "$OUT/dominant_probe.json")
fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_timed" -o run -- \
  python3 $ROOT/bench.py --no-cpu-baseline --no-stage-profile --timed-kernel $TIMED --batch $BATCH --steps 40 --warmup 3 $ONLY \
  > "$OUT/trace_timed_bench.json" 2> "$OUT/trace_timed.err"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run -- python3 $SHORT \
  > /dev/null 2> "$OUT/pmc_fetch.err"
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run -- python3 $SHORT \
  > /dev/null 2> "$OUT/pmc_write.err"
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
  SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --output-format csv -d "$OUT/pmc_sq_a" -o run -- python3 $SHORT \
  > /dev/null 2> "$OUT/pmc_sq_a.err"
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT \
  SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM SQ_WAIT_INST_LDS --output-format csv -d "$OUT/pmc_sq_b" -o run \
  -- python3 $SHORT > /dev/null 2> "$OUT/pmc_sq_b.err"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/calib_fetch" -o run -- \
  $ROOT/tools/pmc_calib > "$OUT/calib_bytes.csv" 2> "$OUT/calib_fetch.err"
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/calib_write" -o run -- \
  $ROOT/tools/pmc_calib > /dev/null 2> "$OUT/calib_write.err"
python3 $ROOT/tools/pmc_calib.py "$OUT" > /dev/null
cd "$ROOT"
python3 tools/pmc_traffic.py "$OUT/pmc_fetch/run_counter_collection.csv" "$OUT/pmc_write/run_counter_collection.csv" $BATCH 1280 720 "$OUT/pmc_traffic.json" > /dev/null
cp "$OUT/pmc_traffic.json" profiles/pmc_traffic.json  # the bench line below reads it
python3 tools/pmc_agg.py "$OUT/pmc_sq_a/run_counter_collection.csv" "$OUT/pmc_sq_b/run_counter_collection.csv" > "$OUT/sq_counters_agg.txt"
python3 tools/timed_launches.py "$OUT/trace_timed/run_kernel_trace.csv" "$OUT/trace_timed_bench.json" > "$OUT/timed_launches.json"
timeout -k 10 400 python3 bench.py --batch $BATCH --timed-kernel $TIMED > "$OUT/bench.json" 2> "$OUT/bench.err"
find "$OUT" -name "*.csv" | sort
