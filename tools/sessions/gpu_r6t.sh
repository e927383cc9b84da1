#!/bin/bash
# Round 6, call t: the materialising queue keeps each record's id in LDS (the flush reads
# only the states) -- parity, C3 A/B against re-reading the id (rid).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6t; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_potmmcp.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/parity.log 2>&1 || { echo parity-failed; tail -40 $O/parity.log; exit 1; }
tail -1 $O/parity.log
for v in cur rid cur rid; do
  lib=""; [ $v != cur ] && lib=$PWD/variants/lib_$v.so
  POMCP_LIB_PATH=$lib timeout -k 10 300 python -u bench.py --env PursuitEvasion-v1 --update-step --steps 3 --warmup 1 --no-cpu-baseline --no-sub > $O/c3_$v.log 2>&1 || { echo c3-failed $v; tail -30 $O/c3_$v.log; exit 1; }
  python - $O/c3_$v.log $v <<'PY'
import json, sys
r = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], round(r["value"] / 1e9, 4), "G", round(r["ms_per_step"], 1), "ms/step update",
      round(r.get("update_ms", -1), 1), "kernel", round(r["roofline"]["kernel_ms"], 1))
PY
done
