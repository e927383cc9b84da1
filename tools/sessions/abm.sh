set -o pipefail
O=gpurun_out/abm_$1; mkdir -p $O; shift
ARGS="$1"; shift
for n in "$@"; do
  echo "== $n" >> $O/exp.log
  POMCP_LIB_PATH=$PWD/variants/lib_$n.so timeout -k 10 300 python bench.py $ARGS --no-cpu-baseline >> $O/exp.log 2>&1 || exit 1
done
grep -E "^==|^\{" $O/exp.log | python3 -c "
import sys,json
for l in sys.stdin:
    if l.startswith('=='): n=l.split()[1]
    else:
        d=json.loads(l); print(n, round(d['value']/1e9,4), 'G', d['roofline'].get('kernel_ms'), 'ms', round(d['roofline']['frac'],4))"
