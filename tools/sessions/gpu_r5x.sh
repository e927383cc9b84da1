#!/bin/bash
# Round 5: per-kernel times of the update()-inclusive PursuitEvasion step with
# the 16-wave log kernels (in-tree library); the visits atomics' ceiling
# (abv: k_compact_log without its per-record visits atomic -- wrong visits).
set -o pipefail
O=gpurun_out/r5x; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o pe -- python3 bench.py --env PursuitEvasion-v1 --trees 32768 --update-step --no-cpu-baseline --no-sub --steps 3 --warmup 1 > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); cut -c1-150 $f | head -14
for v in cur abv cur abv; do
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
