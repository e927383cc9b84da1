# bench per library (run via gpurun): tools/exp_bench.sh OUT "bench args" lib...
set -o pipefail
O=gpurun_out/$1; A=$2; shift 2
mkdir -p $O
for lib in "$@"; do
  echo "== $lib" >> $O/exp.log
  POMCP_LIB_PATH=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --steps 2 $A >> $O/exp.log 2>&1 || exit 1
done
