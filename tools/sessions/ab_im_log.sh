#!/bin/bash
# A/B (via gpurun): I-NTMCP with a level's log record stored after the next level's
# record loads.  The -DIM_LOG_DEFER patch was measured (-1%) and reverted: re-apply
# it to simulate() before running this; otherwise both builds are equal.
set -o pipefail
mkdir -p gpurun_out/imlog
for v in "base:" "defer:-DIM_LOG_DEFER"; do
  n=${v%%:*}; f=${v#*:}
  POMCP_LIB_PATH=/tmp/lib_$n.so POMCP_EXTRA_FLAGS="$f" \
    python -c "import sys; sys.path.insert(0,'posggym-baselines_amd'); from posggym_baselines_amd import build; build.build(force=True, verbose=False)" || exit 1
done
POMCP_LIB_PATH=/tmp/lib_defer.so timeout -k 10 600 python -u -m pytest tests/test_gpu_intmcp.py -x -q --timeout 200 --timeout-method thread > gpurun_out/imlog/parity_defer.log 2>&1
echo parity rc=$?; tail -1 gpurun_out/imlog/parity_defer.log
for r in 1 2 3; do
for n in base defer; do
  POMCP_LIB_PATH=/tmp/lib_$n.so timeout -k 10 200 python bench.py --planner intmcp --no-cpu-baseline > gpurun_out/imlog/$n.log 2>&1 || exit 1
  echo $n $(grep -h '^{' gpurun_out/imlog/$n.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(round(d['value']/1e9,4), round(d['roofline']['kernel_ms'],2))")
done
done
