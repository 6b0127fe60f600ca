# concurrent throughput vs detector instances (batches in flight), interleaved, at the
# driver's 20-step window and at 100 steps: gpurun_out/$TAG/instances.txt
set -o pipefail
TAG=${TAG:-inst}; O=gpurun_out/$TAG; mkdir -p $O
for r in 1 2; do for st in 20 100; do for i in 4 5 6; do
  echo -n "round=$r steps=$st instances=$i " >> $O/instances.txt
  timeout -k 10 200 python3 bench.py --instances $i --steps $st --no-cpu-baseline --latency-frames 0 --host-ingest-steps 0 \
    --c3-latency-iters 0 --node-path-calls 0 --no-stage-profile --no-kernel-timer --isolated-batches 0 2>>$O/err.txt | python3 -c "
import json,sys; j=json.load(sys.stdin); print(j['value'])" >> $O/instances.txt || exit 1
done; done; done
