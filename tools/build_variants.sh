#!/bin/bash
# Build A/B / ablation variants of the engine into variants/lib_NAME.so (CPU side).
#   tools/build_variants.sh "name:FLAGS" ...      (FLAGS: extra -D options, may be empty)
# Up to 3 builds run at once (each compiles its two units in parallel).
set -o pipefail
mkdir -p variants
pids=()
for v in "$@"; do
  n=${v%%:*}; f=${v#*:}
  ( POMCP_LIB_PATH=$PWD/variants/lib_$n.so POMCP_EXTRA_FLAGS="$f" \
      python -c "import sys; sys.path.insert(0,'posggym-baselines_amd'); from posggym_baselines_amd import build; build.build(force=True, verbose=False)" \
      > /tmp/bv_$n.log 2>&1 && echo "built $n" || { echo "FAILED $n"; tail -5 /tmp/bv_$n.log; } ) &
  pids+=($!)
  if [ ${#pids[@]} -ge 3 ]; then wait ${pids[0]}; pids=("${pids[@]:1}"); fi
done
wait
