#!/bin/bash
# Round 6, call n: k_search's unit under other LLVM scheduling strategies (the
# headline, Driving-v1 65,536 x 65,536), interleaved with the current library.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6n; mkdir -p $O
for v in cur maxilp maxmem ilpunr ilptrk cur maxilp maxmem ilpunr ilptrk; do
  lib=""; [ $v != cur ] && lib=$PWD/variants/lib_$v.so
  POMCP_LIB_PATH=$lib timeout -k 10 200 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-sub > $O/h_$v.log 2>&1 || { echo failed $v; tail -20 $O/h_$v.log; exit 1; }
  python - $O/h_$v.log $v <<'PY'
import json, sys
r = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], round(r["value"] / 1e9, 4), "G", round(r["ms_per_step"], 1), "ms/step kernel", round(r["roofline"]["kernel_ms"], 1), "frac", round(r["roofline"]["frac"], 4))
PY
done
echo done
