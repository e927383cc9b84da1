#!/bin/bash
# A/B of the update kernels on the PursuitEvasion update()-inclusive step:
#   tools/ab_update.sh TAG "tests to run (pytest -k expr or '')" lib1 lib2 ...
# (variants/lib_<name>.so; the in-tree library runs the tests)
set -o pipefail
export TMPDIR=/tmp
T=$1; K=$2; shift 2
O=gpurun_out/abu_$T; mkdir -p $O
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$K" > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
  tail -1 $O/test.log
fi
for n in "$@" "$@"; do
  echo "== $n" >> $O/exp.log
  POMCP_LIB_PATH=$PWD/variants/lib_$n.so timeout -k 10 300 python bench.py --no-cpu-baseline --no-sub --steps 2 --warmup 1 --env ${ENV:-PursuitEvasion-v1} --update-step --trees ${TREES:-32768} >> $O/exp.log 2>&1 || exit 1
done
python3 - $O/exp.log <<'PY'
import json, sys
name = None
for line in open(sys.argv[1]):
    if line.startswith("=="):
        name = line.split()[1]
    elif line.startswith("{"):
        d = json.loads(line)
        print(f"{name:8s} {d['value']/1e9:6.3f} G sims/s  ms/step {d['ms_per_step']:8.1f} kernel {d['roofline']['kernel_ms']:8.1f} ms update_ms {d.get('update_ms')}")
PY
