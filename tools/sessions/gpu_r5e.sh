#!/bin/bash
# Round 5: A/B of where the simulation-aligned blocks are computed (sim start
# in registers / LDS-held words / speculatively in the root level's shadow),
# then lane-kernel parity of each variant.
set -o pipefail
O=gpurun_out/r5e; mkdir -p $O
for n in align spec ldsw specl align spec ldsw specl; do
  echo "== $n" >> $O/exp.log
  POMCP_LIB_PATH=$PWD/variants/lib_$n.so timeout -k 10 300 python bench.py --no-cpu-baseline --no-sub --steps 3 --warmup 1 >> $O/exp.log 2>&1 || exit 1
done
grep -E "^==|^\{" $O/exp.log | python3 -c "
import sys,json
for l in sys.stdin:
    if l.startswith('=='): n=l.split()[1]
    else:
        d=json.loads(l); print(n, round(d['value']/1e9,5), 'G', round(d['roofline'].get('kernel_ms'),2), 'ms', round(d['roofline']['frac'],4))"
for n in spec ldsw specl; do
  POMCP_LIB_PATH=$PWD/variants/lib_$n.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_mcts_policies.py tests/test_gpu_potmmcp.py -k "lane or mcts or potmmcp" -x -q --timeout 300 --timeout-method thread > $O/parity_$n.log 2>&1 || { echo "parity $n FAILED"; tail -20 $O/parity_$n.log; exit 1; }
  echo "parity $n: $(tail -1 $O/parity_$n.log)"
done
echo done
