#!/bin/bash
# Ablation builds of k_search (measurement only; results are NOT the reference's):
# how much of a search the Philox RNG, the FP64 UCB scoring, the belief
# particle line and the particle-log stores cost.  Any other library can be
# compared too: put it at variants/lib_NAME.so and list NAME in VARIANTS.
#   tools/ablate.sh build      (here: hipcc the variants into variants/)
#   tools/ablate.sh run TAG    (GPU box, via gpurun)
set -o pipefail
if [ "$1" = build ]; then
  mkdir -p variants
  for v in "base:" "philox3:-DPB_PHILOX_ROUNDS=3" "nosel:-DPOMCP_ABLATE_SELECT" \
           "nobelief:-DPOMCP_ABLATE_BELIEF" "nolog:-DPOMCP_ABLATE_LOG" \
           "nocutslot:-DPOMCP_ABLATE_CUTSLOT"; do
    n=${v%%:*}; f=${v#*:}
    POMCP_LIB_PATH=$PWD/variants/lib_$n.so POMCP_EXTRA_FLAGS="$f" \
      python -c "import sys; sys.path.insert(0,'posggym-baselines_amd'); from posggym_baselines_amd import build; build.build(force=True)" || exit 1
  done
  exit 0
fi
O=gpurun_out/ablate_$2
mkdir -p $O
for n in ${VARIANTS:-base philox3 nosel nobelief nolog base}; do
  echo "== $n" >> $O/exp.log
  POMCP_LIB_PATH=$PWD/variants/lib_$n.so timeout -k 10 300 python bench.py --no-cpu-baseline --no-sub --steps 2 --warmup 1 >> $O/exp.log 2>&1 || exit 1
done
python3 - $O/exp.log <<'PY'
import json, sys
name = None
for line in open(sys.argv[1]):
    if line.startswith("=="):
        name = line.split()[1]
    elif line.startswith("{"):
        d = json.loads(line)
        print(f"{name:8s} {d['value']/1e9:6.3f} G sims/s  kernel {d['roofline']['kernel_ms']:8.1f} ms")
PY
