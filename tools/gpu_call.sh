# one GPU call of this session: GPU tests of the tree, interleaved A/B of library
# builds, extra bench legs, B = 1 latency breakdowns
set -o pipefail
O=gpurun_out/${TAG:-c2}; mkdir -p $O
# a failing test is recorded and the call goes on; a crash, abort or time limit ends it
fatal() { case $1 in 0|1) return 0;; *) echo "fatal rc=$1" >> $O/fatal.txt; exit $1;; esac; }
if [ -n "${GPU_TESTS:-}" ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1; fatal $?
fi
if [ -n "${PAR_LIB:-}" ]; then
  AT_HIP_LIB=$PAR_LIB timeout -k 10 300 python -u -m pytest tests/test_stream_parity.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $O/parity.log 2>&1; fatal $?
fi
if [ -n "${LAT_LIBS:-}" ]; then
  for lib in $LAT_LIBS; do
    echo "== $lib" >> $O/lat.txt
    AT_HIP_LIB=$lib timeout -k 10 120 python tools/lat_stages.py 300 >> $O/lat.txt 2>&1 || exit 1
    AT_HIP_LIB=$lib timeout -k 10 120 python tools/latency_phases.py 1 >> $O/lat.txt 2>&1 || exit 1
  done
fi
if [ -n "${LAT_ENVS:-}" ]; then
  for r in 1 2; do for ev in $LAT_ENVS; do
    echo "== $ev" >> $O/lat_env.txt
    env AT_HIP_LIB=${AT_HIP_LIB:-ros_vision_amd/ab/libat_hip_exp.so} $ev timeout -k 10 120 python tools/lat_stages.py 300 2>&1 | grep wall >> $O/lat_env.txt || exit 1
  done; done
fi
if [ -n "${C3_ENVS:-}" ]; then
  for r in 1 2; do for ev in $C3_ENVS; do
    echo -n "round=$r $ev " >> $O/c3_env.txt
    env AT_HIP_LIB=${AT_HIP_LIB:-ros_vision_amd/ab/libat_hip_exp.so} $ev timeout -k 10 200 python bench.py --steps 10 --no-cpu-baseline --no-stage-profile --host-ingest-steps 0 --latency-frames 500 \
      2>>$O/err.txt | python3 -c "import json,sys; j=json.load(sys.stdin); print(j['p50_latency_ms'], j['p50_latency_hbm_ms'], j['p50_latency_c3_ms'])" >> $O/c3_env.txt || exit 1
  done; done
fi
if [ -n "${PROFILE:-}" ]; then bash tools/profile_round.sh $PROFILE > /dev/null || exit 1; fi
if [ -n "${PHASE_LIBS:-}" ]; then
  for lib in $PHASE_LIBS; do
    echo "== $lib B=${PHASE_B:-128}" >> $O/phases.txt
    AT_HIP_LIB=$lib timeout -k 10 120 python tools/latency_phases.py ${PHASE_B:-128} 2>&1 | grep -v amdgpu >> $O/phases.txt || exit 1
  done
fi
if [ -n "${LIBS:-}" ]; then TAG=${TAG:-c2} bash tools/ab_stages.sh > /dev/null || exit 1; fi
if [ -n "${LIBS1080:-}" ]; then
  for r in 1 2; do for lib in $LIBS1080; do
    echo -n "round=$r lib=$lib " >> $O/ab1080.txt
    AT_HIP_LIB=$lib timeout -k 10 200 python bench.py --width 1920 --height 1080 --tags 24 --steps 40 --no-cpu-baseline --latency-frames 200 \
      --host-ingest-steps 0 --c3-latency-iters 0 --no-kernel-timer 2>>$O/err.txt | python3 -c "
import json,sys; j=json.load(sys.stdin); print(j['value'], j['p50_latency_hbm_ms'], j['detections_per_frame'], ' '.join('%s=%.4f' % kv for kv in j['stage_ms_per_batch'].items()))" >> $O/ab1080.txt || exit 1
  done; done
fi
if [ -n "${PSTOPS:-}" ]; then TAG=${TAG:-c2}/abl STOPS=0 PSTOPS="$PSTOPS" bash tools/ablate.sh > /dev/null || exit 1; fi
if [ -n "${EXTRA_LEGS:-}" ]; then
  timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --ingest scatter --no-cpu-baseline --latency-frames 0 --host-ingest-steps 0 --c3-latency-iters 0 > $O/bench_scatter_n1.json 2> $O/scatter.err || exit 1
  timeout -k 10 240 python bench.py --width 1920 --height 1080 --tags 24 --no-cpu-baseline --host-ingest-steps 0 --c3-latency-iters 0 > $O/bench_1080p.json 2> $O/bench_1080p.err || exit 1
fi
