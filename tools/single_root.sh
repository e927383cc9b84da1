# Single-root and B-sweep measurements, run via
# gpurun: tools/single_root.sh TAG
set -o pipefail
O=gpurun_out/$1
mkdir -p $O
B="timeout -k 10 300 python bench.py --no-cpu-baseline --steps 3 --warmup 1"
$B --trees 1 --sims 65536 > $O/b1_exact.log 2>&1 && \
$B --trees 64 --root-parallel 64 --sims 1024 > $O/rp64.log 2>&1 && \
$B --trees 1024 --root-parallel 1024 --sims 64 > $O/rp1024.log 2>&1 && \
$B --trees 16384 --root-parallel 16384 --sims 4 > $O/rp16384.log 2>&1 && \
$B --trees 64 --sims 65536 > $O/b64.log 2>&1 && \
$B --trees 1024 --sims 65536 > $O/b1024.log 2>&1 && \
$B --trees 16384 --sims 65536 > $O/b16384.log 2>&1 && \
$B --deep --trees 16384 --sims 4096 --max-blocks 4160 > $O/deep.log 2>&1
rc=$?
for f in $O/*.log; do echo "$f: $(tail -1 $f | python -c 'import json,sys
try:
  d=json.loads(sys.stdin.read()); print("%.4g sims/s  %.3f ms/step  frac=%.3f" % (d["value"], d["ms_per_step"], d["roofline"]["frac"]))
except Exception as e: print("ERR", e)')"; done
exit $rc
