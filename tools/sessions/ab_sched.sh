#!/bin/bash
# A/B (via gpurun): LLVM scheduler strategies on the exact single tree (k_search_lds)
set -o pipefail
mkdir -p gpurun_out/sched
for v in "base:" "ilp:-mllvm -amdgpu-sched-strategy=max-ilp" "iter:-mllvm -amdgpu-sched-strategy=iterative-ilp" "o2:-O2"; do
  n=${v%%:*}; f=${v#*:}
  POMCP_LIB_PATH=/tmp/lib_$n.so POMCP_EXTRA_FLAGS="$f" \
    python -c "import sys; sys.path.insert(0,'posggym-baselines_amd'); from posggym_baselines_amd import build; build.build(force=True, verbose=False)" > gpurun_out/sched/build_$n.log 2>&1 || { echo "build $n failed"; continue; }
done
for r in 1 2; do
for n in base ilp iter o2; do
  [ -f /tmp/lib_$n.so ] || continue
  POMCP_LIB_PATH=/tmp/lib_$n.so timeout -k 10 120 python bench.py --trees 1 --sims 65536 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/sched/$n.log 2>&1 || exit 1
  echo $n $(grep -h '^{' gpurun_out/sched/$n.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(round(d['value']), d['ms_per_step'])")
done
done
