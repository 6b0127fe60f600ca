set -uo pipefail
OUT=$(pwd)/gpurun_out/cfg1; mkdir -p $OUT
for r in 1 2 3; do
for cfg in "4 128 8" "4 256 8" "3 256 8" "2 256 8"; do
  read -r inst batch hwq <<< "$cfg"
  echo -n "round=$r inst=$inst batch=$batch " >> $OUT/r.txt
  timeout -k 10 150 python3 bench.py --instances $inst --batch $batch --hw-queues $hwq --pool 128 --steps $((32000 / batch)) --warmup 5 --no-cpu-baseline --latency-frames 0 --no-stage-profile --no-kernel-timer 2>>$OUT/err.txt | python3 -c "import json,sys; j=json.load(sys.stdin); print(j['value'], j['ms_per_step'])" >> $OUT/r.txt || exit 1
done; done
