#!/bin/bash
# Round 6, call v: k_log_filter's visits summed over a chunk (call u hung in the
# first re-root test; the mid-chunk flush's vused read now precedes a barrier):
# one re-root test under a short limit first, then parity, vf0 parity and the
# C3 A/B against one atomic per node and segment (segvis).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6v; mkdir -p $O
timeout -k 10 100 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "test_gpu_matches_reference_goldens and lane-c1_ucb" --timeout 80 --timeout-method thread > $O/one.log 2>&1 || { echo one-failed; tail -30 $O/one.log; exit 1; }
grep -E "PASSED|FAILED" $O/one.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_potmmcp.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/parity.log 2>&1 || { echo parity-failed; tail -30 $O/parity.log; exit 1; }
tail -1 $O/parity.log
POMCP_LIB_PATH=$PWD/variants/lib_vf0.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "full_size_reroot or forced_small_arena" --timeout 200 --timeout-method thread > $O/parity_vf0.log 2>&1 || { echo parity-vf0-failed; tail -30 $O/parity_vf0.log; exit 1; }
tail -1 $O/parity_vf0.log
for v in cur segvis cur segvis; do
  lib=""; [ $v != cur ] && lib=$PWD/variants/lib_$v.so
  POMCP_LIB_PATH=$lib timeout -k 10 300 python -u bench.py --env PursuitEvasion-v1 --update-step --steps 3 --warmup 1 --no-cpu-baseline --no-sub > $O/c3_$v.log 2>&1 || { echo c3-failed $v; tail -30 $O/c3_$v.log; exit 1; }
  python - $O/c3_$v.log $v <<'PY'
import json, sys
r = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], round(r["value"] / 1e9, 4), "G", round(r["ms_per_step"], 1), "ms/step update",
      round(r.get("update_ms", -1), 1), "kernel", round(r["roofline"]["kernel_ms"], 1))
PY
done
