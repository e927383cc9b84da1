#!/bin/bash
# Registers, scratch, LDS and occupancy of the search kernels as the compiler
# allocates them (gfx950 device compile of the library's single translation unit).
# usage: tools/resource_usage.sh   (CPU only; prints one line per search kernel)
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -fPIC -I"$R/include" \
  -c --cuda-device-only -Rpass-analysis=kernel-resource-usage \
  "$R/posggym-baselines_amd/csrc/pomcp_capi.hip" -o /tmp/pomcp_ru.o 2>&1 |
python3 -c "
import re, sys
cur, rows = None, {}
for l in sys.stdin:
    m = re.search(r'remark:\s+(Function Name|VGPRs|AGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]): (\S+)', l)
    if not m: continue
    k, v = m.groups()
    if k == 'Function Name': cur = v; rows[cur] = {}
    else: rows[cur][k.split()[0]] = v
for f, r in rows.items():
    if 'k_search' in f or 'k_im_search' in f:
        print(f, r)
"
