#!/bin/bash
# usage (via gpurun): bash tools/ablate_wave.sh -> gpurun_out/st5/
# ablations of the exact single tree (measurement builds in /tmp; results wrong)
set -o pipefail
mkdir -p gpurun_out/st5
for v in base:"" nosel:"-DPB_ABL_NOSEL" nolog:"-DPB_ABL_NOLOG" both:"-DPB_ABL_NOSEL -DPB_ABL_NOLOG"; do
  n=${v%%:*}; f=${v#*:}
  POMCP_LIB_PATH=/tmp/lib_$n.so POMCP_EXTRA_FLAGS="$f" \
    python -c "import sys; sys.path.insert(0,'posggym-baselines_amd'); from posggym_baselines_amd import build; build.build(force=True, verbose=False)" || exit 1
done
for r in 1 2; do
for n in base nosel nolog both; do
  POMCP_LIB_PATH=/tmp/lib_$n.so timeout -k 10 120 python bench.py --trees 1 --sims 65536 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/st5/$n.log 2>&1 || exit 1
  echo $n $(grep -h '^{' gpurun_out/st5/$n.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(round(d['value']), d['ms_per_step'])")
done
done
