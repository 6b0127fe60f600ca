#!/bin/bash
# Per-kernel HBM bytes (FETCH_SIZE / WRITE_SIZE, separate rocprofv3 --pmc passes)
# of library variants: LIBS="a.so b.so" TAG=pab bash tools/pmc_ab.sh
set -euo pipefail
TAG=${TAG:-pab}; ROOT=$(pwd); OUT=$ROOT/gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
# (only the timed loop's batches: the latency, C3, host-ingest, node and isolated legs
# would add dispatches at other batch sizes to the per-frame averages)
SHORT="$ROOT/bench.py --no-cpu-baseline --no-stage-profile --batch 192 --steps 4 --warmup 1 --latency-frames 0 --host-ingest-steps 0 --c3-latency-iters 0 --node-path-calls 0 --isolated-batches 0"
for lib in $LIBS; do
  n=$(basename $lib .so)
  cd /tmp
  AT_HIP_LIB=$ROOT/$lib timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/$n/f" -o run -- python3 $SHORT > /dev/null 2> "$OUT/$n.ferr"
  AT_HIP_LIB=$ROOT/$lib timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/$n/w" -o run -- python3 $SHORT > /dev/null 2> "$OUT/$n.werr"
  cd $ROOT
  python3 tools/pmc_traffic.py "$OUT/$n/f/run_counter_collection.csv" "$OUT/$n/w/run_counter_collection.csv" 192 1280 720 "$OUT/$n.json" > /dev/null
done
python3 - "$OUT" $LIBS <<'PY'
import json, os, sys
out = sys.argv[1]
for lib in sys.argv[2:]:
    n = os.path.basename(lib)[:-3]
    d = json.load(open(os.path.join(out, n + ".json")))
    print(n, "raw %.2f MB/frame corrected %.2f" % (d["raw_fetch_plus_write_per_frame"] / 1e6, d["hbm_bytes_per_frame"] / 1e6),
          " ".join("%s=%.2f/%.2f" % (k, v["fetch_bytes_per_frame"] / 1e6, v["write_bytes_per_frame"] / 1e6)
                   for k, v in sorted(d["kernels"].items())))
PY
