#!/bin/bash
# round-4 step c: the late step-tree hand-off test, k_search ablations on the
# current code, and a kernel profile of the update()-inclusive PursuitEvasion step
set -o pipefail
O=gpurun_out/r4c; mkdir -p $O
export TMPDIR=/tmp
POMCP_LIB_PATH=$PWD/variants/lib_cur2.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "late_step_tree or overflow_map" -q --timeout 200 --timeout-method thread > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -2 $O/test.log
for n in cur2 philox3 nosel nolog cur2 philox3; do
  echo "== $n" >> $O/exp.log
  POMCP_LIB_PATH=$PWD/variants/lib_$n.so timeout -k 10 300 python bench.py --no-cpu-baseline --no-sub --steps 3 --warmup 1 >> $O/exp.log 2>&1 || exit 1
done
python3 - $O/exp.log <<'PY'
import json, sys
name = None
for line in open(sys.argv[1]):
    if line.startswith("=="):
        name = line.split()[1]
    elif line.startswith("{"):
        d = json.loads(line)
        print(f"{name:8s} {d['value']/1e9:6.3f} G sims/s  kernel {d['roofline']['kernel_ms']:8.1f} ms frac {d['roofline']['frac']:.4f}")
PY
POMCP_LIB_PATH=$PWD/variants/lib_cur2.so timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_pe -o run -- python3 bench.py --env PursuitEvasion-v1 --update-step --no-cpu-baseline --steps 2 --warmup 1 --trees 16384 > $O/prof_pe.log 2>&1 || { tail -20 $O/prof_pe.log; exit 1; }
find $O/prof_pe -type f ! -name '*kernel_stats.csv' -delete
cat $O/prof_pe/run_kernel_stats.csv | cut -c1-160
tail -c 600 $O/prof_pe.log
