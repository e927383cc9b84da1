#!/bin/bash
# Round 6, call p: the materialising pass reading child slots 0-1 first (lazy)
# and skipping the overflow-insert stage's barriers when no thread needs it
# (oskip): C3 A/B, the pass's section timing, parity of the combined variant.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6p; mkdir -p $O
POMCP_LIB_PATH=$PWD/variants/lib_both.so timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_potmmcp.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/parity_both.log 2>&1 || { echo parity-failed; tail -40 $O/parity_both.log; exit 1; }
tail -1 $O/parity_both.log
for v in cur lazy oskip both cur lazy oskip both; do
  lib=""; [ $v != cur ] && lib=$PWD/variants/lib_$v.so
  POMCP_LIB_PATH=$lib timeout -k 10 300 python -u bench.py --env PursuitEvasion-v1 --update-step --steps 3 --warmup 1 --no-cpu-baseline --no-sub > $O/c3_$v.log 2>&1 || { echo c3-failed $v; tail -30 $O/c3_$v.log; exit 1; }
  python - $O/c3_$v.log $v <<'PY'
import json, sys
r = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], round(r["value"] / 1e9, 4), "G", round(r["ms_per_step"], 1), "ms/step update",
      round(r.get("update_ms", -1), 1), "kernel", round(r["roofline"]["kernel_ms"], 1))
PY
done
POMCP_LIB_PATH=$PWD/variants/lib_clogtb.so timeout -k 10 300 python -u tools/clog_timing.py --trees 65536 > $O/timing_clogtb.txt 2>&1 || { echo timing-failed; tail -20 $O/timing_clogtb.txt; exit 1; }
cat $O/timing_clogtb.txt
echo done
