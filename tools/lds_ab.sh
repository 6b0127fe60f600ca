#!/bin/bash
# LDS bank conflicts per kernel of library variants (one SQ --pmc pass each, no
# traces): LIBS="a.so b.so" TAG=lab bash tools/lds_ab.sh
set -euo pipefail
TAG=${TAG:-lab}; ROOT=$(pwd); OUT=$ROOT/gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
SHORT="$ROOT/bench.py --no-cpu-baseline --no-stage-profile --batch 128 --steps 4 --warmup 1 --latency-frames 0"
for lib in $LIBS; do
  n=$(basename $lib .so)
  cd /tmp
  AT_HIP_LIB=$ROOT/$lib timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE \
    SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
    --output-format csv -d "$OUT/$n" -o run -- python3 $SHORT > /dev/null 2> "$OUT/$n.err"
  cd $ROOT
  echo "== $n" >> $OUT/lds.txt
  python3 tools/pmc_agg.py "$OUT/$n/run_counter_collection.csv" >> $OUT/lds.txt
done
python3 - $OUT/lds.txt <<'PY'
import re, sys
lib = k = None; d = {}
for line in open(sys.argv[1]):
    if line.startswith("=="):
        lib = line.split()[1]; k = None; continue
    if " dispatches=" in line:  # (kernel names hold spaces: k_blob<256, 4096, false>)
        k = line.split(" dispatches=")[0]; d[(lib, k)] = {}; continue
    p = line.split()
    if len(p) == 2 and k:
        d[(lib, k)][p[0]] = float(p[1])
for (lib, k), c in sorted(d.items(), key=lambda t: (t[0][1], t[0][0])):
    n = c.get("SQ_INSTS_LDS", 0)
    if n:
        print("%-40s %-16s lds=%10.0f conflict/op=%.3f salu=%10.0f valu=%10.0f" % (
            k[-40:], lib, n, c.get("SQ_LDS_BANK_CONFLICT", 0) / n, c.get("SQ_INSTS_SALU", 0), c.get("SQ_INSTS_VALU", 0)))
PY
