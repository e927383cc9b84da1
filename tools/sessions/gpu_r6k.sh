#!/bin/bash
# Round 6, call k: the materialising pass waits for the previous chunk's flag
# atomics just before its own (not at the end of each chunk): parity, C3 A/B
# against the old placement, and the pass's section timing (diagnostics builds).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6k; mkdir -p $O
timeout -k 10 240 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "full_size_reroot" --timeout 200 --timeout-method thread > $O/probe.log 2>&1 || { echo probe-failed; tail -40 $O/probe.log; exit 1; }
tail -3 $O/probe.log
timeout -k 10 1000 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_potmmcp.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo suite-failed; tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
for v in cur fend cur fend; do
  lib=""; [ $v != cur ] && lib=$PWD/variants/lib_$v.so
  POMCP_LIB_PATH=$lib timeout -k 10 300 python -u bench.py --env PursuitEvasion-v1 --update-step --steps 3 --warmup 1 --no-cpu-baseline --no-sub > $O/c3_$v.log 2>&1 || { echo c3-failed $v; tail -30 $O/c3_$v.log; exit 1; }
  python - $O/c3_$v.log $v <<'PY'
import json, sys
r = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], round(r["value"] / 1e9, 4), "G", round(r["ms_per_step"], 1), "ms/step update",
      round(r.get("update_ms", -1), 1), "kernel", round(r["roofline"]["kernel_ms"], 1), r["config"]["trees_per_gpu"])
PY
done
for v in clogt clogtf; do
  echo "== $v"
  POMCP_LIB_PATH=$PWD/variants/lib_$v.so timeout -k 10 300 python -u tools/clog_timing.py --trees 65536 > $O/timing_$v.txt 2>&1 || { echo timing-failed; tail -20 $O/timing_$v.txt; exit 1; }
  cat $O/timing_$v.txt
done
echo done
