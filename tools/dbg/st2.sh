set -o pipefail
mkdir -p gpurun_out/st2
export POMCP_LIB_PATH=$PWD/posggym-baselines_amd/posggym_baselines_amd/_lib/libpomcp_hip_dbg.so
timeout -k 10 60 python bench.py --trees 1 --sims 256 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/st2/b1_small.log 2>&1
echo rc=$?
tail -c 3000 gpurun_out/st2/b1_small.log
