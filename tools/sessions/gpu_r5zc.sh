#!/bin/bash
# Round 5: k_compact_log x / A by a multiply (dv4, dv3, dv2: 4 / 3 / 2 records
# per thread per pass) vs km3 (the LDS kept counts, 3 records per thread) and
# the in-tree library (cur), update()-inclusive PursuitEvasion step; GPU
# parity of dv3.
set -o pipefail
O=gpurun_out/r5zc; mkdir -p $O
for v in cur km3 dv3 dv4 dv2 cur km3 dv3 dv4 dv2; do
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
POMCP_LIB_PATH=$PWD/variants/lib_dv3.so timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_potmmcp.py -x -q --timeout 300 --timeout-method thread > $O/parity.log 2>&1 || { echo "parity FAILED"; grep -E "FAILED|Error|assert" $O/parity.log | head -20; tail -30 $O/parity.log; exit 1; }
echo "parity dv3: $(tail -1 $O/parity.log)"
echo done
