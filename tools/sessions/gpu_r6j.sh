#!/bin/bash
# Round 6, call j: packed block maps for the filter (k_pack_cmap), 32-segment chunks; A/B of
# chunk sizes 16 / 64 and the materialising pass at 6 / 8 waves per SIMD.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6j; mkdir -p $O
timeout -k 10 240 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "full_size_reroot and lane-" --timeout 120 --timeout-method thread > $O/probe.log 2>&1 || { echo probe-failed; tail -40 $O/probe.log; exit 1; }
tail -3 $O/probe.log
timeout -k 10 1000 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_potmmcp.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo suite-failed; tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
for v in cur ch16 ch64 wpe6 wpe8; do
  lib=""; [ $v != cur ] && lib=$PWD/variants/lib_$v.so
  POMCP_LIB_PATH=$lib timeout -k 10 300 python -u bench.py --env PursuitEvasion-v1 --update-step --steps 3 --warmup 1 --no-cpu-baseline --no-sub > $O/c3_$v.log 2>&1 || { echo c3-failed $v; tail -30 $O/c3_$v.log; exit 1; }
  python - $O/c3_$v.log $v <<'PY'
import json, sys
r = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], round(r["value"] / 1e9, 4), "G", round(r["ms_per_step"], 1), "ms/step update",
      round(r.get("update_ms", -1), 1), "kernel", round(r["roofline"]["kernel_ms"], 1), r["config"]["trees_per_gpu"])
PY
done
P=$O/prof_c3; mkdir -p $P
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $P/trace -o run -- python3 bench.py --env PursuitEvasion-v1 --update-step --steps 3 --warmup 1 --no-cpu-baseline --no-sub > $P/c3_trace.log 2>&1 || { echo prof-failed; tail -20 $P/c3_trace.log; exit 1; }
find $P -type f ! -name '*kernel_stats.csv' ! -name '*.log' -delete
cat $(find $P -name '*kernel_stats.csv') | cut -c1-220 | head -12
echo done
