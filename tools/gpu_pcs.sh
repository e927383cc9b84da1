#!/bin/bash
# PC sampling (host trap) of k_search on a short bench run of a -gline-tables-only
# build (same code; PCs map to source lines): where the wave's time goes.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/pcs; mkdir -p $O
POMCP_LIB_PATH=$PWD/variants/lib_dbg.so timeout -k 10 240 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time --pc-sampling-interval 1 --output-format csv -d $O/raw -o run -- python3 bench.py --no-cpu-baseline --no-sub --sims 4096 --steps 1 --warmup 1 > $O/bench.log 2>&1 || { echo pcs-failed; tail -20 $O/bench.log; ls -R $O | head; exit 1; }
ls -R $O | head -20
f=$(find $O/raw -name '*pc_sampling*' | head -1)
echo "file: $f"; head -3 "$f"
python3 - "$f" > $O/pcs_summary.txt <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
print("rows", len(rows), "cols", list(rows[0].keys()) if rows else None)
by = collections.Counter()
for r in rows:
    k = (r.get("Instruction_Comment") or "") + " | " + (r.get("Instruction") or "")
    by[k] += 1
for k, c in by.most_common(400):
    print(c, k)
PY
head -50 $O/pcs_summary.txt
find $O/raw -type f -size +20M -delete
echo done
