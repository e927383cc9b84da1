#!/bin/bash
# Round 5: k_compact_log kept counts by one LDS atomic per record instead of 6-ballot lane groups (km4; km3 = also 3 records per thread per pass) vs the in-tree library (cur)
set -o pipefail
O=gpurun_out/r5zb; mkdir -p $O
for v in cur km4 km3 cur km4 km3; do
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
