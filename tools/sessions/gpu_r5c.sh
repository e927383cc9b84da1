#!/bin/bash
# Round 5 diagnostics of k_search: parity of the new base, A/B of the obs-key
# skip at deferred levels, ablations, phase timing, SQ counters.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5c; mkdir -p $O
POMCP_LIB_PATH=$PWD/variants/lib_base.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "lane" -x -q --timeout 300 --timeout-method thread > $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }
tail -1 $O/parity.log
for n in base nocutskip base nocutskip philox3 nosel nolog; do
  echo "== $n" >> $O/exp.log
  POMCP_LIB_PATH=$PWD/variants/lib_$n.so timeout -k 10 300 python bench.py --no-cpu-baseline --no-sub --steps 3 --warmup 1 >> $O/exp.log 2>&1 || exit 1
done
grep -E "^==|^\{" $O/exp.log | python3 -c "
import sys,json
for l in sys.stdin:
    if l.startswith('=='): n=l.split()[1]
    else:
        d=json.loads(l); print(n, round(d['value']/1e9,4), 'G', round(d['roofline'].get('kernel_ms'),1), 'ms', round(d['roofline']['frac'],4))"
PT_PREBUILT=$PWD/variants/lib_timing.so timeout -k 10 300 python tools/phase_timing.py --sims 4096 > $O/phase.log 2>&1 || { tail -20 $O/phase.log; exit 1; }
cat $O/phase.log | tail -25
run() {  # name counters...
  local name=$1; shift
  POMCP_LIB_PATH=$PWD/variants/lib_base.so timeout -k 10 300 rocprofv3 --pmc "$@" --output-format csv -d $O/$name -o run -- python3 bench.py --no-cpu-baseline --no-sub --sims 8192 --steps 1 --warmup 1 > $O/$name.log 2>&1 || { echo "pass $name failed"; exit 1; }
}
run p1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_BRANCH
run p2 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS
find $O -name '*counter_collection.csv' | while read f; do python3 - "$f" <<'PY'
import csv, sys
from collections import defaultdict
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "k_search" in r.get("Kernel_Name", "")]
acc = defaultdict(float)
for r in rows[-1:]:
    pass
last = {}
for r in rows:
    last[r["Counter_Name"]] = (r.get("Dispatch_Id"), float(r["Counter_Value"]))
# sum per counter over the last dispatch id
did = max(int(r["Dispatch_Id"]) for r in rows)
for r in rows:
    if int(r["Dispatch_Id"]) == did:
        acc[r["Counter_Name"]] += float(r["Counter_Value"])
print(sys.argv[1].split('/')[-3], dict(acc))
PY
done > $O/pmc_summary.txt
cat $O/pmc_summary.txt
find $O -type f ! -name '*.log' ! -name '*.txt' -delete
echo done
