#!/bin/bash
# Round 5: k_compact_log section timing after the fused extraction and the
# visits table (PB_CLOG_TIMING build), and records per thread per pass 3 / 2
# vs 4 at 16 waves, update()-inclusive PursuitEvasion step.
set -o pipefail
O=gpurun_out/r5za; mkdir -p $O
POMCP_LIB_PATH=$PWD/variants/lib_clogt.so timeout -k 10 300 python tools/clog_timing.py --trees 32768 > $O/clog.txt 2>&1 || { tail -20 $O/clog.txt; exit 1; }
grep -v amdgpu.ids $O/clog.txt
for v in cur lr3 lr2 cur lr3 lr2; do
  lib=""; [ $v != cur ] && lib=$PWD/variants/lib_$v.so
  echo "== $v" >> $O/ab.log
  POMCP_LIB_PATH=$lib timeout -k 10 300 python bench.py --env PursuitEvasion-v1 --trees 32768 --update-step --no-cpu-baseline --no-sub --steps 3 --warmup 1 >> $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
done
grep -E "^==|^\{" $O/ab.log | python3 -c "
import sys,json
for l in sys.stdin:
    if l.startswith('=='): n=l.strip()
    else:
        d=json.loads(l); print(n, round(d['value']/1e9,4), 'G', round(d['ms_per_step'],1), 'ms/step', 'update', round(d.get('update_ms', 0), 1), 'search', round(d['roofline']['kernel_ms'], 1))"
echo done
