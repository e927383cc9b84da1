#!/bin/bash
# Round 5: (1) records per thread per pass of k_extract / k_compact_log (2 / 4 / 8)
# on the update()-inclusive PursuitEvasion step; (2) phase timing of the exact
# single tree's search wave (k_search_lds, one tree x 65,536 sims).
set -o pipefail
O=gpurun_out/r5m; mkdir -p $O
for v in cur lr8 lr2 cur lr8 lr2; do
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
PT_PREBUILT=$PWD/variants/lib_pt.so timeout -k 10 300 python tools/phase_timing.py --trees 1 --sims 65536 --kernel wave > $O/pt_wave.txt 2>&1 || { tail -20 $O/pt_wave.txt; exit 1; }
grep -v amdgpu.ids $O/pt_wave.txt
echo done
