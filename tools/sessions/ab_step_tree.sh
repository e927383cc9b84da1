#!/bin/bash
# usage (via gpurun): bash tools/ab_step_tree.sh -> gpurun_out/st7/
# A/B of the step-tree producer / slot counts (measurement builds in /tmp)
set -o pipefail
mkdir -p gpurun_out/st7
for v in "base:" "np1:-DPB_SPEC_PRODUCERS=1 -DPB_SPEC_SLOTS=2 -DPB_SPEC_POOL_KB=132" "np3:-DPB_SPEC_PRODUCERS=3 -DPB_SPEC_SLOTS=4 -DPB_SPEC_POOL_KB=124"; do
  n=${v%%:*}; f=${v#*:}
  POMCP_LIB_PATH=/tmp/lib_$n.so POMCP_EXTRA_FLAGS="$f" \
    python -c "import sys; sys.path.insert(0,'posggym-baselines_amd'); from posggym_baselines_amd import build; build.build(force=True, verbose=False)" || exit 1
done
for r in 1 2; do
for n in base np1 np3; do
  POMCP_LIB_PATH=/tmp/lib_$n.so timeout -k 10 120 python bench.py --trees 1 --sims 65536 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/st7/$n.log 2>&1 || exit 1
  echo $n $(grep -h '^{' gpurun_out/st7/$n.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(round(d['value']), d['ms_per_step'])")
done
done
