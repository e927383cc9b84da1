"""k_im_search phase breakdown (diagnostics; run on the GPU box).

Builds a diagnostics copy of the engine with -DPOMCP_PHASE_TIMING into /tmp,
runs warm searches of the bench's I-NTMCP workload and prints the share of
lane time per section of a simulation (each mark drains outstanding memory
operations, so a section is charged the waits of the loads it issued).

    python tools/phase_timing_im.py [--pairs B --sims S]
"""
import argparse
import ctypes as C
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = "/tmp/libpomcp_hip_timing.so"
os.environ["POMCP_LIB_PATH"] = LIB
sys.path[:0] = [ROOT, os.path.join(ROOT, "posggym-baselines_amd")]
NAMES = ["sim start (root particle, start view)", "level: selection", "level: other agent's action",
         "level: step + obs keys", "level: child lookups", "level: descend (view, log, path)",
         "leaf expansion", "rollout", "backup", "sim end", "-", "-"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=16384)
    ap.add_argument("--sims", type=int, default=256)
    ap.add_argument("--env", default="Driving-v1")
    args = ap.parse_args()
    env = dict(os.environ, POMCP_EXTRA_FLAGS="-DPOMCP_PHASE_TIMING")
    subprocess.run([sys.executable, "-c", "from posggym_baselines_amd import build; build.build(force=True)"],
                   check=True, env=env, cwd=os.path.join(ROOT, "posggym-baselines_amd"))
    import numpy as np
    from posggym_baselines_amd import _native as N
    from posggym_baselines_amd.envs import DrivingModel, PursuitEvasionModel
    from posggym_baselines_amd.planning import BatchedINTMCP, MCTSConfig
    from posggym_baselines_amd.planning.intmcp import plan_intmcp_capacities
    import bench
    cfg = MCTSConfig(seed=0, num_sims=args.sims, **dict(bench.TEST_CFG, state_belief_only=False))
    model = PursuitEvasionModel() if args.env == "PursuitEvasion-v1" else DrivingModel()
    A = model.action_spaces["0"].n
    caps = plan_intmcp_capacities(cfg, model.spec.max_episode_steps, args.sims, 3, A)
    bp = BatchedINTMCP(model, "0", cfg, args.pairs, args.sims, capacities=caps)
    bp.init_synthetic(1000)
    bp.search(fetch=False)                      # warm: the trees of a second search
    fn = N.load().intmcp_debug_phase_timing
    cnt = C.c_int32()
    assert fn(bp.engine._ctx, None, 0, C.byref(cnt)) == 0
    bp.search(fetch=False)
    assert fn(bp.engine._ctx, None, 0, C.byref(cnt)) == 0
    buf = np.zeros(cnt.value, dtype=np.uint64)
    assert fn(bp.engine._ctx, buf.ctypes.data_as(C.c_void_p), cnt.value, C.byref(cnt)) == 0
    per = buf.reshape(-1, 12).astype(np.float64)
    per = per[per.sum(1) > 0]
    tot = per.sum(0)
    sims = 2 * args.sims
    print(f"{args.env}: {len(per)} pairs; s_memtime ticks per pair per simulation:")
    for i, n in enumerate(NAMES):
        if n != "-":
            print(f"  {n:40s} {tot[i] / len(per) / sims:9.2f}  {100 * tot[i] / tot.sum():5.1f}%")
    print(f"  {'total':40s} {tot.sum() / len(per) / sims:9.2f}")
    bp.close()


if __name__ == "__main__":
    main()
