# round-5 GPU call: GPU tests, counter list, default bench line, isolated-only traced run
# usage: bash tools/r05_call.sh TAG
set -o pipefail
TAG=${1:-r05a}; O=gpurun_out/$TAG; mkdir -p $O
R=$(pwd)
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc" > $O/rc.txt
case $rc in 0|1) ;; *) exit $rc;; esac
if [ -n "${LIST:-}" ]; then timeout -k 10 60 rocprofv3 -L > $O/counters.txt 2>&1 || true; fi
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || exit 1
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/trace_iso -o run -- python3 $R/bench.py --isolated-only > $R/$O/iso_traced.json 2> $R/$O/iso_traced.err) || exit 1
python3 tools/roofline_check.py $O/trace_iso/run_kernel_stats.csv $O/bench.json $O/iso_traced.json > $O/roofline_check.json
