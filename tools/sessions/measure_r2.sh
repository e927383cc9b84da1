# Round-2 measurements (run via gpurun): headline bench (with the CPU
# baseline), config 3, config 5, single-root modes, then rocprof profiles of
# the headline and of I-NTMCP (fixed arenas: every launch the main workload).
# usage: tools/measure_r2.sh TAG
set -o pipefail
T=$1
O=gpurun_out/m_$T
mkdir -p $O
B="timeout -k 10 400 python bench.py"
$B > $O/bench.log 2>&1 && \
$B --env PursuitEvasion-v1 --no-cpu-baseline > $O/bench_pe.log 2>&1 && \
$B --planner intmcp --no-cpu-baseline > $O/bench_im.log 2>&1 && \
$B --trees 1024 --root-parallel 1024 --sims 64 --no-cpu-baseline > $O/bench_rp1024.log 2>&1 && \
$B --trees 1 --sims 65536 --steps 2 --no-cpu-baseline > $O/bench_b1.log 2>&1 && \
bash tools/profile.sh $T && \
bash tools/profile.sh ${T}_intmcp --planner intmcp --no-cpu-baseline --arena 2845,3537,4811 && \
bash tools/pmc_im.sh $T --arena 2845,3537,4811
