#!/bin/bash
# A/B of two builds inside one gpurun call (same box):
#   tools/ab.sh TAG BASE NEW "BENCH ARGS" "PYTEST ARGS"
# variants/lib_BASE.so and variants/lib_NEW.so; the parity tests run on NEW.
set -o pipefail
O=gpurun_out/ab_$1; mkdir -p $O
if [ -n "$5" ]; then
  POMCP_LIB_PATH=$PWD/variants/lib_$3.so timeout -k 10 600 python -u -m pytest $5 -x -q \
    --timeout 300 --timeout-method thread > $O/test.log 2>&1 || { tail -20 $O/test.log; exit 1; }
  tail -1 $O/test.log
fi
for n in $2 $3 $2 $3; do
  echo "== $n" >> $O/exp.log
  POMCP_LIB_PATH=$PWD/variants/lib_$n.so timeout -k 10 300 python bench.py $4 --no-cpu-baseline \
    >> $O/exp.log 2>&1 || exit 1
done
grep -E "^==|^\{" $O/exp.log | python3 -c "
import sys,json
for l in sys.stdin:
    if l.startswith('=='): n=l.split()[1]
    else:
        d=json.loads(l); print(n, round(d['value']/1e9,4), 'G', d['roofline'].get('kernel_ms'), 'ms', round(d['roofline']['frac'],4))"
