#!/bin/bash
# Round 6, call q: tiers of the materialising pass's lazy child-slot reads
# (lazyAB: A slots first, then B, then the rest; lazy = 2 then the rest): C3 A/B
# and re-root parity of the 1-1-rest variant.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6q; mkdir -p $O
POMCP_LIB_PATH=$PWD/variants/lib_lazy11.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "reroot or compaction or episode or defer or batched" --timeout 300 --timeout-method thread > $O/parity_lazy11.log 2>&1 || { echo parity-failed; tail -40 $O/parity_lazy11.log; exit 1; }
tail -1 $O/parity_lazy11.log
for v in cur lazy lazy1 lazy11 lazy12 lazy21 cur lazy lazy1 lazy11 lazy12 lazy21; do
  lib=""; [ $v != cur ] && lib=$PWD/variants/lib_$v.so
  POMCP_LIB_PATH=$lib timeout -k 10 300 python -u bench.py --env PursuitEvasion-v1 --update-step --steps 3 --warmup 1 --no-cpu-baseline --no-sub > $O/c3_$v.log 2>&1 || { echo c3-failed $v; tail -30 $O/c3_$v.log; exit 1; }
  python - $O/c3_$v.log $v <<'PY'
import json, sys
r = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], round(r["value"] / 1e9, 4), "G", round(r["ms_per_step"], 1), "ms/step update",
      round(r.get("update_ms", -1), 1), "kernel", round(r["roofline"]["kernel_ms"], 1))
PY
done
echo done
