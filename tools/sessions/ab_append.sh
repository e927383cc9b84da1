#!/bin/bash
# A/B (via gpurun): k_search with the particle-log record appended inside the
# level (after the child-line loads, LDS-counter positions) -- parity on the
# lane kernel with that build, then the headline bench alternating.
set -o pipefail
mkdir -p gpurun_out/app
for v in "base:" "mid:-DPB_APPEND_MID"; do
  n=${v%%:*}; f=${v#*:}
  POMCP_LIB_PATH=/tmp/lib_$n.so POMCP_EXTRA_FLAGS="$f" \
    python -c "import sys; sys.path.insert(0,'posggym-baselines_amd'); from posggym_baselines_amd import build; build.build(force=True, verbose=False)" || exit 1
done
POMCP_LIB_PATH=/tmp/lib_mid.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "lane" > gpurun_out/app/parity_mid.log 2>&1
echo parity rc=$?; tail -1 gpurun_out/app/parity_mid.log
for r in 1 2 3; do
for n in base mid; do
  POMCP_LIB_PATH=/tmp/lib_$n.so timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/app/$n.log 2>&1 || exit 1
  echo $n $(grep -h '^{' gpurun_out/app/$n.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(round(d['value']/1e9,4), round(d['roofline']['kernel_ms'],1))")
done
done
