# k_quad_fin in isolation (one detector instance: kernels serialized), with and without
# its accepted-quad appends (blob stop 5, experiment build), product library beside
set -o pipefail
R=$(pwd); O=gpurun_out/${TAG:-r06q}; mkdir -p $O; export TMPDIR=/tmp
run() {  # $1 = name, $2 = library, $3 = blob stop
  (cd /tmp && AT_HIP_LIB=$2 AT_DIAG_BLOB_STOP=$3 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/$1 -o run -- \
    python3 $R/bench.py --instances 1 --steps 20 --no-cpu-baseline --no-stage-profile --latency-frames 0 --host-ingest-steps 0 \
    --c3-latency-iters 0 --node-path-calls 0 --isolated-batches 0 --no-kernel-timer > $R/$O/$1.json 2> $R/$O/$1.err) || exit 1
}
run prod $R/ros_vision_amd/libat_hip.so 0
run exp0 $R/ros_vision_amd/ab/libat_hip_exp.so 0
run exp5 $R/ros_vision_amd/ab/libat_hip_exp.so 5
run base $R/ros_vision_amd/ab/libat_base.so 0
