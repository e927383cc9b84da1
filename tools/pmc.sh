#!/bin/bash
# SQ / TCC counter passes for k_search (run on the GPU box via gpurun).
# usage: tools/pmc.sh TAG [bench args...]
TAG=${1:-x}; shift || true
ARGS="$@"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_$TAG
mkdir -p $OUT
run() {  # name counters...
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$name -o run -- python3 bench.py --no-cpu-baseline $ARGS > $OUT/$name.log 2>&1 || { echo "pass $name failed"; exit 1; }
}
run p1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_BRANCH
run p2 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS
run p3 GRBM_GUI_ACTIVE SQ_INSTS_VALU_FP64 SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS TCC_HIT_sum TCC_MISS_sum
echo pmc-done
