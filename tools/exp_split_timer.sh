TAG=pe3; ROOT=$(pwd); OUT=$ROOT/gpurun_out/$TAG; mkdir -p $OUT
B="$ROOT/bench.py --no-cpu-baseline --no-stage-profile --latency-frames 0 --steps 40 --warmup 3"
summ() { python3 -c "import json,sys; j=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(j['value'], j['roofline']['avg_launch_ms'], j['roofline']['kernel'])"; }
run() { echo -n "$1: " >> $OUT/r.txt; shift; timeout -k 10 120 "$@" 2>>$OUT/err.txt | summ >> $OUT/r.txt || exit 1; }
timeout -k 10 200 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || exit 1
run "split-graph ktimer" python3 $B
run "no ktimer" python3 $B --no-kernel-timer
timeout -k 10 200 python3 bench.py --no-cpu-baseline > $OUT/bench_default.json 2>>$OUT/err.txt
