# Round-6 end-of-session evidence in one GPU call (the profile round ran separately,
# profiles/r06k): GPU tests + smoke of the tree, the B=1 kernel chain (rocprofv3 kernel
# trace of tools/lat_trace.py), the 1920x1080 100-step line and the scatter topology at
# world size 1 beside the local loop.  usage: bash tools/r06_final.sh TAG
set -o pipefail
TAG=${1:-r06end}; O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/lat_trace -o run -- python3 $GRAFT_REPO_ROOT/tools/lat_trace.py 300 > /dev/null 2>&1) || exit 1
python3 tools/gap_report.py $O/lat_trace/run_kernel_trace.csv > $O/lat_gaps.txt || exit 1
timeout -k 10 300 python bench.py --width 1920 --height 1080 --tags 24 --steps 100 --no-cpu-baseline --host-ingest-steps 0 --c3-latency-iters 0 --node-path-calls 0 --latency-frames 300 > $O/bench_1080p_100steps.json 2> $O/bench_1080p.err || exit 1
LEG="--no-cpu-baseline --latency-frames 0 --host-ingest-steps 0 --c3-latency-iters 0 --node-path-calls 0"
timeout -k 10 240 python bench.py $LEG > $O/bench_local_n1.json 2> $O/local.err || exit 1
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --ingest scatter $LEG > $O/bench_scatter_n1.json 2> $O/scatter.err || exit 1
echo ok > $O/done.txt
