#!/bin/bash
# HBM traffic and SQ counters of the re-root kernels in the C3 update()-inclusive
# step (k_compact, k_pack_cmap, k_log_filter, the materialising pass); one
# counter pass per rocprofv3 run.  usage: tools/sessions/pmc_update.sh TAG
TAG=${1:-x}
export TMPDIR=/tmp
OUT=gpurun_out/pmcu_$TAG
mkdir -p $OUT
ARGS="--env PursuitEvasion-v1 --update-step --steps 2 --warmup 1 --no-cpu-baseline --no-sub"
run() {  # name counters...
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$name -o run -- python3 bench.py $ARGS > $OUT/$name.log 2>&1 || { echo "pass $name failed"; tail -5 $OUT/$name.log; exit 1; }
}
run fetch FETCH_SIZE
run write WRITE_SIZE
run p1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_BUSY_CYCLES
run p2 SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE
find $OUT -type f ! -name '*counter_collection.csv' ! -name '*.log' -delete
python3 tools/update_pmc.py $OUT
