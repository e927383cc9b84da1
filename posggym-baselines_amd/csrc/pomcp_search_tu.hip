// k_search (pomcp_search.hip) in a translation unit of its own.
//
// The tree-per-lane search is compiled with LLVM's iterative ILP machine
// scheduler (build.py kSearchFlags), which schedules its phase loop +2% faster
// on the Driving-v1 headline than the default scheduler, while the same flag
// costs the I-NTMCP search 5% -- so only this unit gets it.
// The shared device code is compiled here inside a namespace of its own so the
// non-template kernels of pomcp_kernels.hip do not collide with the C-ABI
// unit's; pomcp_capi.hip launches the instantiations pb_search_kernel returns.
#include <hip/hip_runtime.h>

#include <climits>
#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstring>

#define PB_SEARCH_TU 1
#define pb pb_search
#include "pomcp_kernels.hip"
#include "pomcp_search.hip"
