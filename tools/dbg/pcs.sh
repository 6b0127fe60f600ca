# PC sampling (rocprofv3 beta) of the k_pre + k_thr_ccl part of the bench loop
set -o pipefail
O=$(pwd)/gpurun_out/pcs; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 -L > $O/list.txt 2>&1 || true
grep -i -A20 "pc sampling\|pc_sampling" $O/list.txt | head -60 > $O/pcs_configs.txt || true
AT_HIP_LIB=$GRAFT_REPO_ROOT/ros_vision_amd/ab/libat_hip_exp.so AT_DIAG_PIPE_STOP=2 timeout -s KILL 150 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method ${METHOD:-stochastic} --pc-sampling-unit ${UNIT:-cycles} --pc-sampling-interval ${IVL:-65536} --output-format csv -d $O/run -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 2 --no-cpu-baseline --latency-frames 0 --host-ingest-steps 0 --c3-latency-iters 0 --no-kernel-timer --no-stage-profile --node-path-calls 0 > $O/bench.json 2> $O/err.txt
echo rc=$? >> $O/err.txt
find $O -type f | head -20
