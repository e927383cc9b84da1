# GPU parity tests + default bench (run via gpurun): tools/gpu_check.sh TAG [bench args]
set -o pipefail
O=gpurun_out/$1; shift
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/bench.log 2>&1
rc=$?; tail -3 $O/gpu_tests.log; tail -1 $O/bench.log | cut -c1-200; exit $rc
