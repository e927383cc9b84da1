# A/B of the step-tree producer count (measurement builds in /tmp)
set -o pipefail
mkdir -p gpurun_out/st4
for v in "3 4 124" "5 6 116" "7 8 108" "2 3 128"; do
  set -- $v
  L=/tmp/lib_np$1.so
  POMCP_LIB_PATH=$L POMCP_EXTRA_FLAGS="-DPB_SPEC_PRODUCERS=$1 -DPB_SPEC_SLOTS=$2 -DPB_SPEC_POOL_KB=$3" \
    python -c "import sys; sys.path.insert(0,'posggym-baselines_amd'); from posggym_baselines_amd import build; build.build(force=True, verbose=False)" || exit 1
done
for r in 1 2; do
for v in 3 5 7 2; do
  POMCP_LIB_PATH=/tmp/lib_np$v.so timeout -k 10 120 python bench.py --trees 1 --sims 65536 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/st4/np$v.log 2>&1 || exit 1
  echo np$v $(grep -h '^{' gpurun_out/st4/np$v.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(round(d['value']), d['ms_per_step'])")
done
done
