#!/bin/bash
# Round 5: fast UCB scores with one Newton step per reciprocal (nr1) and a
# reciprocal-based sqrt(log N) (s): error of the reciprocals, A/B of the
# headline and I-NTMCP, then parity of nr1s (goldens, lane tests, exact fallback).
set -o pipefail
O=gpurun_out/r5n; mkdir -p $O
for v in cur nr1 nr1s nr2s; do
  lib=""; [ $v != cur ] && lib=$PWD/variants/lib_$v.so
  POMCP_LIB_PATH=$lib timeout -k 10 120 python tools/recip_err.py >> $O/err.log 2>&1 || { tail -20 $O/err.log; exit 1; }
done
cat $O/err.log | grep -v amdgpu.ids
for v in cur nr1 nr1s nr2s cur nr1 nr1s nr2s; do
  lib=""; [ $v != cur ] && lib=$PWD/variants/lib_$v.so
  echo "== $v" >> $O/ab.log
  POMCP_LIB_PATH=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --no-sub --steps 3 --warmup 1 >> $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
done
for v in cur nr1s cur nr1s; do
  lib=""; [ $v != cur ] && lib=$PWD/variants/lib_$v.so
  echo "== im $v" >> $O/ab.log
  POMCP_LIB_PATH=$lib timeout -k 10 300 python bench.py --planner intmcp --no-cpu-baseline --no-sub --steps 5 --warmup 1 >> $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
done
grep -E "^==|^\{" $O/ab.log | python3 -c "
import sys,json
for l in sys.stdin:
    if l.startswith('=='): n=l.strip()
    else:
        d=json.loads(l); r=d['roofline']; print(n, round(d['value']/1e9,4), 'G', round(r['kernel_ms'],2), 'ms', round(r['frac'],4))"
POMCP_LIB_PATH=$PWD/variants/lib_nr1s.so timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_mcts_policies.py tests/test_gpu_potmmcp.py tests/test_gpu_intmcp.py -x -q -k "not reciprocals" --timeout 300 --timeout-method thread > $O/parity.log 2>&1 || { echo "parity FAILED"; grep -E "FAILED|Error|assert" $O/parity.log | head -20; tail -30 $O/parity.log; exit 1; }
echo "parity: $(tail -1 $O/parity.log)"
echo done
