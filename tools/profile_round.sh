#!/bin/bash
# One GPU call collecting this round's profiles (MI355X_MICROARCH.md HBM/rocprofv3):
#   1. the plain bench line (bench.json)
#   2. rocprofv3 --kernel-trace --stats of `bench.py --isolated-only` (every launch
#      serialized: each kernel's rocprof average is its isolated duration) and
#      tools/roofline_check.py: the line's roofline frac recomputed from it
#   3. rocprofv3 --kernel-trace --stats of the timed loop (concurrent launches) and
#      tools/timed_launches.py: the DOMINANT kernel's traced launches vs the live timer
#   4. FETCH_SIZE and WRITE_SIZE, each in its own --pmc pass (never with traces)
#   5. SQ counter passes (8 SQ counters + GRBM_GUI_ACTIVE each): stall shares, LDS,
#      per-class VALU instruction counts; tools/valu_rates (issue cost per class) and
#      tools/valu_ceiling.py
#   6. FETCH_SIZE / WRITE_SIZE passes over tools/pmc_calib (known byte counts per
#      access width, for the gfx950 correction)
# Output: gpurun_out/$TAG/...   usage: bash tools/profile_round.sh TAG [BATCH]
set -euo pipefail
TAG=${1:-prof}
BATCH=${2:-192}
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
ONLY="--latency-frames 0 --host-ingest-steps 0 --c3-latency-iters 0 --node-path-calls 0"
SHORT="$ROOT/bench.py --no-cpu-baseline --no-stage-profile --batch $BATCH --steps 4 --warmup 1 $ONLY --isolated-batches 0"
timeout -k 10 400 python3 bench.py --batch $BATCH > "$OUT/bench.json" 2> "$OUT/bench.err"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_iso" -o run -- \
  python3 $ROOT/bench.py --isolated-only --batch $BATCH > "$OUT/iso_traced.json" 2> "$OUT/iso_traced.err"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_timed" -o run -- \
  python3 $ROOT/bench.py --no-cpu-baseline --no-stage-profile --isolated-batches 0 --batch $BATCH --steps 40 --warmup 3 $ONLY \
  > "$OUT/trace_timed_bench.json" 2> "$OUT/trace_timed.err"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run -- python3 $SHORT \
  > /dev/null 2> "$OUT/pmc_fetch.err"
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run -- python3 $SHORT \
  > /dev/null 2> "$OUT/pmc_write.err"
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
  SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE --output-format csv -d "$OUT/pmc_sq_a" -o run -- python3 $SHORT \
  > /dev/null 2> "$OUT/pmc_sq_a.err"
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT \
  SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d "$OUT/pmc_sq_b" -o run \
  -- python3 $SHORT > /dev/null 2> "$OUT/pmc_sq_b.err"
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 \
  SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT GRBM_GUI_ACTIVE \
  --output-format csv -d "$OUT/pmc_sq_c" -o run -- python3 $SHORT > /dev/null 2> "$OUT/pmc_sq_c.err"
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 \
  SQ_INSTS_VALU_INT32 SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE \
  --output-format csv -d "$OUT/pmc_sq_d" -o run -- python3 $SHORT > /dev/null 2> "$OUT/pmc_sq_d.err"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/calib_fetch" -o run -- \
  $ROOT/tools/pmc_calib > "$OUT/calib_bytes.csv" 2> "$OUT/calib_fetch.err"
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/calib_write" -o run -- \
  $ROOT/tools/pmc_calib > /dev/null 2> "$OUT/calib_write.err"
timeout -k 10 120 $ROOT/tools/valu_rates > "$OUT/valu_rates.jsonl"
cd "$ROOT"
python3 tools/pmc_calib.py "$OUT" > /dev/null
python3 tools/pmc_traffic.py "$OUT/pmc_fetch/run_counter_collection.csv" "$OUT/pmc_write/run_counter_collection.csv" $BATCH 1280 720 "$OUT/pmc_traffic.json" > /dev/null
python3 tools/pmc_agg.py "$OUT/pmc_sq_a/run_counter_collection.csv" "$OUT/pmc_sq_b/run_counter_collection.csv" \
  "$OUT/pmc_sq_c/run_counter_collection.csv" "$OUT/pmc_sq_d/run_counter_collection.csv" > "$OUT/sq_counters_agg.txt"
STEP=$(python3 -c "import json,sys; print(json.load(open(sys.argv[1]))['ms_per_step'])" "$OUT/bench.json")
python3 tools/valu_ceiling.py "$OUT/valu_rates.jsonl" "$OUT/pmc_sq_a/run_counter_collection.csv" \
  "$OUT/pmc_sq_b/run_counter_collection.csv" "$OUT/pmc_sq_c/run_counter_collection.csv" \
  "$OUT/pmc_sq_d/run_counter_collection.csv" --frames=$BATCH --step-ms=$STEP > "$OUT/valu_ceiling.json"
python3 tools/roofline_check.py "$OUT/trace_iso/run_kernel_stats.csv" "$OUT/bench.json" "$OUT/iso_traced.json" > "$OUT/roofline_check.json"
python3 tools/timed_launches.py "$OUT/trace_timed/run_kernel_trace.csv" "$OUT/trace_timed_bench.json" > "$OUT/timed_launches.json"
find "$OUT" -name "*.csv" | sort
