"""k_search phase breakdown (diagnostics; run on the GPU box).

Builds a diagnostics copy of the engine with -DPOMCP_PHASE_TIMING into
/tmp, runs one warm search on the bench workload and prints the share of wave
time per loop section (each mark drains outstanding memory operations, so a
section is charged the waits of the loads it issued).

    python tools/phase_timing.py [--trees B --sims S]
"""
import argparse
import ctypes as C
import math
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.environ.get("PT_PREBUILT") or "/tmp/libpomcp_hip_timing.so"
os.environ["POMCP_LIB_PATH"] = LIB
sys.path[:0] = [ROOT, os.path.join(ROOT, "posggym-baselines_amd")]
NAMES = ["start+root (LDS)", "level: stats line wait", "level: selection",
         "level: child line wait", "level: rest", "rollout", "backup", "loop/other",
         "  step: philox x2", "  step: drv_step2", "  step: reward+done", "  step: obs key",
         "  find_slot", "  slot write / ovf", "  log+path entry", "  (before step)"]
# k_search_lds (--kernel wave): tree 0's sections
NAMES_WAVE = ["start", "level: draws", "level: LDS line", "level: step + obs key",
              "level: log(N) wait", "level: selection", "level: slots / readout",
              "level: log + path + descend", "rollout", "backup", "-", "-", "-", "-", "-", "-"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trees", type=int, default=65536)
    ap.add_argument("--sims", type=int, default=4096)
    ap.add_argument("--kernel", default="lane", choices=["lane", "wave"])
    args = ap.parse_args()
    os.environ["POMCP_SEARCH_KERNEL"] = args.kernel
    if not os.environ.get("PT_PREBUILT"):   # else LIB was built beforehand (on the CPU side)
        env = dict(os.environ, POMCP_EXTRA_FLAGS="-DPOMCP_PHASE_TIMING")
        subprocess.run([sys.executable, "-c", "from posggym_baselines_amd import build; build.build(force=True)"],
                       check=True, env=env, cwd=os.path.join(ROOT, "posggym-baselines_amd"))
    import numpy as np
    from posggym_baselines_amd import _native as N
    from posggym_baselines_amd.envs import DrivingModel
    from posggym_baselines_amd.planning import BatchedPOMCP, MCTSConfig
    from posggym_baselines_amd.planning.engine import plan_capacities
    import bench
    cfg = MCTSConfig(seed=0, num_sims=args.sims, **bench.TEST_CFG)
    model = DrivingModel()
    caps = plan_capacities(cfg, 50, args.sims, 1, reroot=False, max_blocks=512, overflow_slots=1024)
    bp = BatchedPOMCP(model, "0", cfg, args.trees, args.sims, capacities=caps)
    bp.init_synthetic(1000)
    fn = N.load().pomcp_debug_phase_timing
    cnt = C.c_int32()
    assert fn(bp.engine._ctx, None, 0, C.byref(cnt)) == 0
    bp.restore()
    bp.search(fetch=False)
    assert fn(bp.engine._ctx, None, 0, C.byref(cnt)) == 0
    buf = np.zeros(cnt.value, dtype=np.uint64)
    assert fn(bp.engine._ctx, buf.ctypes.data_as(C.POINTER(C.c_uint64)), cnt.value, C.byref(cnt)) == 0
    per = buf.reshape(-1, 16).astype(np.float64)
    per = per[per.sum(1) > 0]
    names = NAMES_WAVE if args.kernel == "wave" else NAMES
    tot = per.sum(0)
    sims = args.sims
    print(f"waves {len(per)}; s_memtime ticks per wave per simulation round:")
    for i, n in enumerate(names):
        print(f"  {n:26s} {tot[i] / len(per) / sims:10.1f}  {100 * tot[i] / tot.sum():5.1f}%")
    print(f"  {'total':26s} {tot.sum() / len(per) / sims:10.1f}")
    bp.close()


if __name__ == "__main__":
    main()
