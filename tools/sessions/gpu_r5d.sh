#!/bin/bash
# Round 5: simulation-aligned step streams -- the whole GPU suite on the new
# library (goldens regenerated from the reference), then A/B against the
# previous base (variants/lib_base.so: per-draw blocks).
set -o pipefail
O=gpurun_out/r5d; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo tests-failed; tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
for n in base align base align; do
  echo "== $n" >> $O/exp.log
  POMCP_LIB_PATH=$PWD/variants/lib_$n.so timeout -k 10 300 python bench.py --no-cpu-baseline --no-sub --steps 3 --warmup 1 >> $O/exp.log 2>&1 || exit 1
done
for n in base align; do
  echo "== pe_$n" >> $O/exp.log
  POMCP_LIB_PATH=$PWD/variants/lib_$n.so timeout -k 10 300 python bench.py --no-cpu-baseline --no-sub --steps 3 --warmup 1 --env PursuitEvasion-v1 >> $O/exp.log 2>&1 || exit 1
  echo "== b1_$n" >> $O/exp.log
  POMCP_LIB_PATH=$PWD/variants/lib_$n.so timeout -k 10 300 python bench.py --no-cpu-baseline --no-sub --steps 3 --warmup 1 --trees 1 >> $O/exp.log 2>&1 || exit 1
done
grep -E "^==|^\{" $O/exp.log | python3 -c "
import sys,json
for l in sys.stdin:
    if l.startswith('=='): n=l.split()[1]
    else:
        d=json.loads(l); print(n, round(d['value']/1e9,5), 'G', round(d['roofline'].get('kernel_ms'),2), 'ms', round(d['roofline']['frac'],4))"
echo done
