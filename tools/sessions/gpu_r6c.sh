#!/bin/bash
# Round 6, call c: Philox4x32-7 streams (fixtures regenerated from the
# reference): the whole GPU suite, then the headline A/B against the same
# library with 10 rounds (variants/lib_p10.so; its results differ, timing only).
set -o pipefail
O=gpurun_out/r6c; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo suite-failed; tail -40 $O/gpu_tests.log; exit 1; }
tail -3 $O/gpu_tests.log
for v in p7 p10 p7 p10; do
  if [ $v = p7 ]; then L=""; else L=$PWD/variants/lib_$v.so; fi
  POMCP_LIB_PATH=$L timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-sub > $O/head_$v.log 2>&1 || { echo head-failed $v; tail -30 $O/head_$v.log; exit 1; }
  python - $O/head_$v.log $v <<'PY'
import json, sys
r = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], round(r["value"] / 1e9, 4), "G", round(r["ms_per_step"], 1), "ms/step kernel",
      round(r["roofline"]["kernel_ms"], 2), "frac", round(r["roofline"]["frac"], 4))
PY
done
echo done
# k_compact_log: 16 waves x 1 workgroup per CU (product) vs 8 waves x 2 (w8, 128 VGPRs)
O=gpurun_out/r6c
for v in w16 w8 w16 w8; do
  if [ $v = w16 ]; then L=""; else L=$PWD/variants/lib_$v.so; fi
  POMCP_LIB_PATH=$L timeout -k 10 300 python -u bench.py --env PursuitEvasion-v1 --update-step --steps 3 --warmup 1 --no-cpu-baseline --no-sub > $O/c3_$v.log 2>&1 || { echo c3-failed $v; tail -30 $O/c3_$v.log; exit 1; }
  python - $O/c3_$v.log $v <<'PY'
import json, sys
r = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], round(r["value"] / 1e9, 4), "G", round(r["ms_per_step"], 1), "ms/step update",
      round(r.get("update_ms", -1), 1), "kernel", round(r["roofline"]["kernel_ms"], 1))
PY
done
for v in clogt clogt8; do
  POMCP_LIB_PATH=$PWD/variants/lib_$v.so timeout -k 10 300 python -u tools/clog_timing.py --trees 32768 > $O/timing_$v.log 2>&1 || { echo timing-failed $v; tail -30 $O/timing_$v.log; exit 1; }
  echo "== $v"; cat $O/timing_$v.log
done
echo done2
