#!/bin/bash
# Round 6, call r: lazy child-slot reads adopted -- the whole GPU suite, the C3
# step, and the materialising pass's section timing with the overflow-map
# lookup count.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6r; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1 || { tail -40 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
timeout -k 10 300 python -u bench.py --env PursuitEvasion-v1 --update-step --steps 3 --warmup 1 --no-cpu-baseline --no-sub > $O/c3.log 2>&1 || { tail -30 $O/c3.log; exit 1; }
python - $O/c3.log <<'PY'
import json, sys
r = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("c3", round(r["value"] / 1e9, 4), "G", round(r["ms_per_step"], 1), "ms/step update", round(r.get("update_ms", -1), 1))
PY
POMCP_LIB_PATH=$PWD/variants/lib_clogtl.so timeout -k 10 300 python -u tools/clog_timing.py --trees 65536 > $O/timing.txt 2>&1 || { tail -20 $O/timing.txt; exit 1; }
cat $O/timing.txt
