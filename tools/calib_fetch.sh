#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration on known access shapes (run via gpurun):
# tools/ubench/randrw.hip reads/writes random 128 B lines of an 8.6 GB buffer
# (far past the 256 MiB Infinity Cache) in k_search's shapes; the counters per
# access against the bytes the kernel moves say what one counted byte means
# for these scattered accesses.  usage: tools/calib_fetch.sh TAG
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/calib_$1
mkdir -p $O
hipcc -O3 --offload-arch=gfx950 -o $O/randrw tools/ubench/randrw.hip || exit 1
timeout -k 10 120 $O/randrw 10 > $O/randrw.log 2>&1 || exit 1
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 180 rocprofv3 --pmc $C --output-format csv -d $O/$C -o run -- $O/randrw 10 > $O/$C.log 2>&1 || exit 1
done
rm -f $O/randrw
python3 tools/calib_summary.py $O
