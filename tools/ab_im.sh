set -o pipefail
O=gpurun_out/ab_$1; mkdir -p $O
POMCP_LIB_PATH=$PWD/variants/lib_$3.so timeout -k 10 300 python -u -m pytest tests/test_gpu_intmcp.py -x -q --timeout 200 --timeout-method thread -k "goldens or batched_pairs" > $O/test.log 2>&1 || exit 1
for n in $2 $3 $2 $3; do
  echo "== $n" >> $O/exp.log
  POMCP_LIB_PATH=$PWD/variants/lib_$n.so timeout -k 10 300 python bench.py --planner intmcp --no-cpu-baseline --steps 3 --warmup 1 >> $O/exp.log 2>&1 || exit 1
done
grep -E "^==|^\{" $O/exp.log | python3 -c "
import sys,json
for l in sys.stdin:
    if l.startswith('=='): n=l.split()[1]
    else:
        d=json.loads(l); print(n, round(d['value']/1e9,4), d['roofline'].get('kernel_ms'))"
