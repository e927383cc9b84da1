#!/bin/bash
# Compare k_search build variants (variants/*.so) on the bench workload.
# usage: tools/exp_variants.sh OUTDIR "trees sims lib" ...
set -o pipefail
OUT=$1; shift
mkdir -p $OUT
for spec in "$@"; do
  set -- $spec
  echo "== trees=$1 sims=$2 lib=$3" >> $OUT/exp.log
  POMCP_LIB_PATH=$3 timeout -k 10 240 python bench.py --trees $1 --sims $2 --steps 2 --warmup 1 --no-cpu-baseline ${@:4} >> $OUT/exp.log 2>&1 || { echo "FAIL $?" >> $OUT/exp.log; exit 1; }
done
echo exp-done
