# Headline measurements of a round (run via gpurun): default bench (with the CPU
# baseline), config 3 (PursuitEvasion-v1), config 5 (I-NTMCP), then the rocprof
# profile of the default bench.  usage: tools/measure_all.sh TAG
set -o pipefail
T=$1
O=gpurun_out/m_$T
mkdir -p $O
timeout -k 10 400 python bench.py > $O/bench.log 2>&1 && \
timeout -k 10 300 python bench.py --env PursuitEvasion-v1 --no-cpu-baseline > $O/bench_pe.log 2>&1 && \
timeout -k 10 300 python bench.py --planner intmcp --no-cpu-baseline > $O/bench_im.log 2>&1 && \
bash tools/profile.sh $T
