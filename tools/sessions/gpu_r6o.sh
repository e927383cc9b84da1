#!/bin/bash
# Round 6, call o: the final library -- the whole GPU suite, smoke, and a short
# headline run (roofline.traffic present: profiles/pmc_search.json is keyed to
# this library).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6o; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1 || { tail -40 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-sub > $O/h.log 2>&1 || { tail -20 $O/h.log; exit 1; }
python - $O/h.log <<'PY'
import json, sys
r = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(round(r["value"] / 1e9, 4), "G frac", round(r["roofline"]["frac"], 4), "traffic", r["roofline"]["traffic"], "lib", r["config"]["lib_sha16"])
PY
