#!/bin/bash
# Round 6, call b: k_compact_log with the wave's cmap staged in LDS and a
# places-only deferred queue; the C3 update()-inclusive step at 65,536 roots
# (two-ended belief region) A/B against the same library classifying from the
# global cmap (variants/lib_nocml.so); then the whole GPU suite.
set -o pipefail
O=gpurun_out/r6b; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "full_size_reroot or pursuit_evasion_batched_reroot or overflow_map or compaction" --timeout 300 --timeout-method thread > $O/reroot_tests.log 2>&1 || { echo tests-failed; tail -40 $O/reroot_tests.log; exit 1; }
tail -2 $O/reroot_tests.log
timeout -k 10 300 python -u tools/c3_footprint.py PursuitEvasion-v1 > $O/footprint.log 2>&1 || { echo probe-failed; tail -30 $O/footprint.log; exit 1; }
cat $O/footprint.log
for v in new nocml new nocml; do
  if [ $v = new ]; then L=""; else L=$PWD/variants/lib_$v.so; fi
  POMCP_LIB_PATH=$L timeout -k 10 300 python -u bench.py --env PursuitEvasion-v1 --update-step --steps 3 --warmup 1 --no-cpu-baseline --no-sub > $O/c3_$v.log 2>&1 || { echo c3-failed $v; tail -30 $O/c3_$v.log; exit 1; }
  python - $O/c3_$v.log $v <<'PY'
import json, sys
r = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], round(r["value"] / 1e9, 4), "G", round(r["ms_per_step"], 1), "ms/step",
      "update", round(r.get("update_ms", -1), 1), "kernel", round(r["roofline"]["kernel_ms"], 1),
      r["config"]["workload"][:90])
PY
done
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo suite-failed; tail -40 $O/gpu_tests.log; exit 1; }
tail -3 $O/gpu_tests.log
echo done
