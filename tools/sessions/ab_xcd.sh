#!/bin/bash
# A/B (via gpurun): k_search with the XCD-aware workgroup -> trees mapping
set -o pipefail
mkdir -p gpurun_out/xcd
for v in "base:" "xcd:-DPB_XCD_REMAP"; do
  n=${v%%:*}; f=${v#*:}
  POMCP_LIB_PATH=/tmp/lib_$n.so POMCP_EXTRA_FLAGS="$f" \
    python -c "import sys; sys.path.insert(0,'posggym-baselines_amd'); from posggym_baselines_amd import build; build.build(force=True, verbose=False)" || exit 1
done
for r in 1 2 3; do
for n in base xcd; do
  POMCP_LIB_PATH=/tmp/lib_$n.so timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/xcd/$n.log 2>&1 || exit 1
  echo $n $(grep -h '^{' gpurun_out/xcd/$n.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(round(d['value']/1e9,4), round(d['roofline']['kernel_ms'],1))")
done
done
