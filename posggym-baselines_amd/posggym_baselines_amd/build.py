"""Build libpomcp_hip.so in-tree with hipcc for gfx950.

    python -m posggym_baselines_amd.build

``-ffp-contract=off`` is required: the reference's FP64 arithmetic (UCB,
Welford, discounting) has no fused multiply-adds and parity is bit-exact.
"""
import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
PROJECT = os.path.dirname(PKG)                       # posggym-baselines_amd/
REPO = os.path.dirname(PROJECT)
CSRC = os.path.join(PROJECT, "csrc")
INCLUDE = os.path.join(REPO, "include")
OUT = os.environ.get("POMCP_LIB_PATH") or os.path.join(PKG, "_lib", "libpomcp_hip.so")
SOURCES = [os.path.join(CSRC, "pomcp_capi.hip")]
SEARCH_SOURCE = os.path.join(CSRC, "pomcp_search_tu.hip")
DEPS = SOURCES + [SEARCH_SOURCE] + [os.path.join(CSRC, f) for f in
                  ("pomcp_kernels.hip", "pomcp_search.hip", "pomcp_search_lds.hip", "pomcp_device.h", "driving.h",
                   "driving_vec.h", "philox.h", "envs.h", "pursuit_evasion.h", "host_exp.h", "host_exp_table.h", "host_api.cpp", "intmcp.hip", "intmcp_capi.hip")] + [
    os.path.join(INCLUDE, "pomcp.h"), os.path.join(INCLUDE, "pomcp_debug.h"),
    os.path.join(INCLUDE, "intmcp.h")]

HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("POMCP_OFFLOAD_ARCH", "gfx950")
FLAGS = ["-O3", "-std=c++17", f"--offload-arch={ARCH}", "-ffp-contract=off", "-fPIC",
         f"-I{INCLUDE}", "-Wall", "-Wno-unused-function"]
# k_search's unit only (pomcp_search_tu.hip): LLVM's iterative ILP scheduler,
# +2% simulations/s on the headline, -5% on k_im_search
SEARCH_FLAGS = (os.environ.get("POMCP_SEARCH_FLAGS") or
                "-mllvm -amdgpu-sched-strategy=iterative-ilp").split()   # env: A/B builds only
# diagnostics builds (e.g. POMCP_EXTRA_FLAGS=-DPOMCP_PHASE_TIMING with a separate
# POMCP_LIB_PATH); never the default library
FLAGS += os.environ.get("POMCP_EXTRA_FLAGS", "").split()


def up_to_date() -> bool:
    if not os.path.exists(OUT):
        return False
    t = os.path.getmtime(OUT)
    return all(os.path.getmtime(d) <= t for d in DEPS if os.path.exists(d))


def build(force: bool = False, verbose: bool = True) -> str:
    if not force and up_to_date():
        return OUT
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    tmp = OUT + ".tmp"
    objs = [tmp + ".capi.o", tmp + ".search.o"]
    cmds = [[HIPCC] + FLAGS + ["-c", "-o", objs[0]] + SOURCES,
            [HIPCC] + FLAGS + SEARCH_FLAGS + ["-c", "-o", objs[1], SEARCH_SOURCE]]
    link = [HIPCC, f"--offload-arch={ARCH}", "-fPIC", "-shared", "-o", tmp] + objs
    if verbose:
        for c in cmds + [link]:
            print(" ".join(c), flush=True)
    # the two units compile in parallel
    procs = [subprocess.Popen(c) for c in cmds]
    rcs = [p.wait() for p in procs]
    for c, rc in zip(cmds, rcs):
        if rc != 0:
            raise subprocess.CalledProcessError(rc, c)
    subprocess.run(link, check=True)
    for o in objs:
        os.remove(o)
    os.replace(tmp, OUT)
    return OUT


if __name__ == "__main__":
    build(force="--force" in sys.argv)
