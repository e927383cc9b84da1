#!/bin/bash
# Round 6, call u: k_log_filter sums the visits over a chunk's segments (one
# atomic per node and chunk) -- parity of the product and of a build flushing
# the table before every segment (vf0), C3 A/B against one atomic per node and
# segment (segvis).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6u; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_potmmcp.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/parity.log 2>&1 || { echo parity-failed; tail -40 $O/parity.log; exit 1; }
tail -1 $O/parity.log
POMCP_LIB_PATH=$PWD/variants/lib_vf0.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "full_size_reroot or forced_small_arena or episode" --timeout 300 --timeout-method thread > $O/parity_vf0.log 2>&1 || { echo parity-vf0-failed; tail -40 $O/parity_vf0.log; exit 1; }
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
