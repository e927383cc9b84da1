#!/bin/bash
# Round 6, call s: the materialising pass skips an absorbing-flag atomic whose
# value the last arrival already sees (on top of the lazy slot reads) -- the
# whole GPU suite, C3 A/B
# against always issuing it (aflag), section timing.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6s; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/parity.log 2>&1 || { echo parity-failed; tail -40 $O/parity.log; exit 1; }
tail -1 $O/parity.log
for v in cur aflag cur aflag; do
  lib=""; [ $v != cur ] && lib=$PWD/variants/lib_$v.so
  POMCP_LIB_PATH=$lib timeout -k 10 300 python -u bench.py --env PursuitEvasion-v1 --update-step --steps 3 --warmup 1 --no-cpu-baseline --no-sub > $O/c3_$v.log 2>&1 || { echo c3-failed $v; tail -30 $O/c3_$v.log; exit 1; }
  python - $O/c3_$v.log $v <<'PY'
import json, sys
r = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], round(r["value"] / 1e9, 4), "G", round(r["ms_per_step"], 1), "ms/step update",
      round(r.get("update_ms", -1), 1), "kernel", round(r["roofline"]["kernel_ms"], 1))
PY
done
POMCP_LIB_PATH=$PWD/variants/lib_clogtf.so timeout -k 10 300 python -u tools/clog_timing.py --trees 65536 > $O/timing.txt 2>&1 || { tail -20 $O/timing.txt; exit 1; }
cat $O/timing.txt
POMCP_LIB_PATH=$PWD/variants/lib_clogtl.so timeout -k 10 300 python -u tools/clog_timing.py --trees 65536 > $O/timing_lazy_only.txt 2>&1 || { tail -20 $O/timing_lazy_only.txt; exit 1; }
cat $O/timing_lazy_only.txt
