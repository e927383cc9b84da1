"""k_compact_log section breakdown (diagnostics; run on the GPU box).

Needs a diagnostics library built with -DPB_CLOG_TIMING (POMCP_LIB_PATH points
at it; build it on the CPU side with
  POMCP_EXTRA_FLAGS=-DPB_CLOG_TIMING POMCP_LIB_PATH=$PWD/variants/lib_clogt.so \
      python -m posggym_baselines_amd.build --force
).  Runs the bench's PursuitEvasion update()-inclusive step once (search,
synthetic env step, update) and prints thread 0's s_memtime ticks per section
per workgroup and the per-workgroup counters.

    python tools/clog_timing.py [--trees B --sims S --env E]
"""
import argparse
import ctypes as C
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "posggym-baselines_amd")]
SECTIONS = ["classify (record, cmap)", "mat: slots + ovf lookup", "mat: serial ovf inserts",
            "mat: flags + fence", "visits, rank, store"]
COUNTERS = ["records", "mat records", "serial ovf records", "flag records", "kept records",
            "overflow-map lookups"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trees", type=int, default=16384)
    ap.add_argument("--sims", type=int, default=65536)
    ap.add_argument("--env", default="PursuitEvasion-v1")
    args = ap.parse_args()
    import numpy as np
    import torch
    from posggym_baselines_amd import _native as N
    from posggym_baselines_amd.envs import DrivingModel, PursuitEvasionModel
    from posggym_baselines_amd.planning import BatchedPOMCP, MCTSConfig
    from posggym_baselines_amd.planning.engine import plan_capacities
    import bench
    cfg = MCTSConfig(seed=0, num_sims=args.sims, **bench.TEST_CFG)
    model = PursuitEvasionModel() if args.env == "PursuitEvasion-v1" else DrivingModel()
    caps = plan_capacities(cfg, model.spec.max_episode_steps, args.sims, 1, reroot=True,
                           max_blocks=512, overflow_slots=1024)
    caps.max_belief = min(caps.max_belief, 70000)
    bp = BatchedPOMCP(model, "0", cfg, args.trees, args.sims, capacities=caps)
    bp.init_synthetic(1000)
    fn = N.load().pomcp_debug_phase_timing
    cnt = C.c_int32()
    assert fn(bp.engine._ctx, None, 0, C.byref(cnt)) == 0
    acts = bp.search()
    obs = bp.engine.synthetic_step(1000, acts)
    t0 = time.perf_counter()
    bp.engine.update(acts, obs)
    print(f"update {1e3 * (time.perf_counter() - t0):.1f} ms")
    assert fn(bp.engine._ctx, None, 0, C.byref(cnt)) == 0
    buf = np.zeros(cnt.value, dtype=np.uint64)
    assert fn(bp.engine._ctx, buf.ctypes.data_as(C.POINTER(C.c_uint64)), cnt.value, C.byref(cnt)) == 0
    per = buf.reshape(-1, 16).astype(np.float64)
    per = per[per[:, 8] > 0]
    print(f"workgroups {len(per)}; per workgroup (mean, s_memtime = shader clock cycles on gfx950):")
    tot = per[:, :5].sum(1)
    for i, n in enumerate(SECTIONS):
        print(f"  {n:28s} {per[:, i].mean() / 1e6:9.2f} Mcycles  {100 * per[:, i].sum() / tot.sum():5.1f}%")
    for i, n in enumerate(COUNTERS):
        print(f"  {n:28s} {per[:, 8 + i].mean():14.0f}")
    passes = per[:, 8].mean() / 1024   # kLogRecs x 256 records per pass
    print(f"  passes {passes:.0f}, ticks per pass {tot.mean() / passes:.0f}")
    bp.close()
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
