#!/bin/bash
# Address-translation and memory-latency counters of k_search (run via gpurun).
# usage: tools/pmc_tlb.sh TAG [bench args...]   -> gpurun_out/tlb_TAG/
TAG=${1:-x}; shift || true
export TMPDIR=/tmp
OUT=gpurun_out/tlb_$TAG
mkdir -p $OUT
run() {  # name counters...
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$name -o run -- python3 bench.py --no-cpu-baseline "${BENCH_ARGS[@]}" > $OUT/$name.log 2>&1 || { echo "pass $name failed"; exit 1; }
}
BENCH_ARGS=("$@")
run t1 TCP_UTCL1_REQUEST_sum TCP_UTCL1_TRANSLATION_MISS_sum
run t2 TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_STALL_MULTI_MISS_sum
run t3 TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum
run t4 TCP_TCC_WRITE_REQ_LATENCY_sum TCP_TCC_WRITE_REQ_sum
run t5 TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum
run t6 GRBM_GUI_ACTIVE GRBM_UTCL2_BUSY
echo tlb-done
