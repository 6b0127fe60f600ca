#!/bin/bash
# One GPU call: rocprofv3 kernel-trace stats of the bench command, then two
# separate PMC passes (FETCH_SIZE, WRITE_SIZE; never combined with traces),
# then the plain bench line.  Output: gpurun_out/$TAG/...
# usage: bash tools/profile_round.sh TAG
set -euo pipefail
TAG=${1:-prof}
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
BENCH="$ROOT/bench.py --no-cpu-baseline --steps 20 --warmup 3 --latency-frames 20"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 $BENCH > "$OUT/trace_bench.json" 2> "$OUT/trace.err"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run -- python3 $ROOT/bench.py --no-cpu-baseline --no-stage-profile --steps 4 --warmup 1 --latency-frames 0 > /dev/null 2> "$OUT/pmc_fetch.err"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run -- python3 $ROOT/bench.py --no-cpu-baseline --no-stage-profile --steps 4 --warmup 1 --latency-frames 0 > /dev/null 2> "$OUT/pmc_write.err"
cd "$ROOT"
timeout -k 10 300 python3 bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
find "$OUT" -name "*.csv" | head -20
# rocprof of the timed-region configuration only (dominant kernel timed live, no
# serialized profile pass, no latency loop): its k_blob average is comparable
# with bench.json's roofline.avg_launch_ms
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_timed" -o run -- python3 $ROOT/bench.py --no-cpu-baseline --no-stage-profile --steps 40 --warmup 3 --latency-frames 0 > "$OUT/trace_timed_bench.json" 2> "$OUT/trace_timed.err"
cd "$ROOT"
