#!/bin/bash
# Round 5 closing library: update()-inclusive step, deferred vs eager cut-off
# lookup (bench.py --defer on/off), 32,768 trees x 65,536 sims, one box.
set -o pipefail
O=gpurun_out/r5zd; mkdir -p $O
run() {  # env defer
  echo "== $1 defer=$2" >> $O/ab.log
  timeout -k 10 300 python bench.py --env $1 --trees 32768 --update-step --defer $2 --no-cpu-baseline --no-sub --steps 3 --warmup 1 >> $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
}
for d in on off on off; do run PursuitEvasion-v1 $d || exit 1; done
for d in on off; do run Driving-v1 $d || exit 1; done
grep -E "^==|^\{" $O/ab.log | python3 -c "
import sys,json
for l in sys.stdin:
    if l.startswith('=='): n=l.strip()
    else:
        d=json.loads(l); print(n, round(d['value']/1e9,4), 'G', round(d['ms_per_step'],1), 'ms/step', 'update', round(d.get('update_ms', 0), 1), 'search', round(d['roofline']['kernel_ms'], 1), d['config']['lib_sha16'])"
echo done
