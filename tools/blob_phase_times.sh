#!/bin/bash
# k_blob phase breakdown: stage times with AT_DIAG_BLOB_STOP=N (diagnostic early exits)
for n in ${STOPS:-1 2 3 4 5 6 0}; do
  echo -n "stop=$n "
  AT_DIAG_BLOB_STOP=$n timeout -k 10 120 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --latency-frames 5 | python -c "import json,sys; j=json.load(sys.stdin); print(j['stage_ms_per_batch'].get('k_blob'), j['stage_ms_per_batch'].get('k_boundary'), j['value'])" || exit 1
done
