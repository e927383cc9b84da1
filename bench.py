"""POMCP simulation throughput on MI355X (BASELINE.json metric).

One step = one exact-mode POMCP search (``get_action``, mcts.py:269-306) of
``--sims`` simulations on each of ``--trees`` synthetic Driving-v1 roots
(tree b's root is the ego's belief after the initial update for
an environment sampled under seed 1000 + b), followed by the root-parallel
exchange: one all-gather (RCCL over xGMI) of every tree's exchange record
((visit count, total value) per root action + step statistics) and the device
merge of every planner's replicas in one fixed order.  Ranks search the same
roots with different RNG keys (seed ^ rank << 32); per-GPU work is fixed as N
grows (weak scaling).  Inputs are resident in HBM before timing starts; each
timed step restores the post-update root state (a few KB per tree) and
re-searches it.

Single-root modes (BASELINE config 2 as ONE planner): ``--trees 1`` is the
exact planner (one tree, one lane); ``--trees K --root-parallel K --sims S/K``
gives one planner K replica trees of S/K simulations each, merged on the
device (``pomcp_merge_roots``), so ``ms_per_step`` is that planner's
``get_action`` latency for S simulations.  ``--deep`` is SURVEY §8(d)'s
rollout-dominated point (gamma 0.99, epsilon 0.01: depth_limit 459).

    python bench.py [--gpus N --steps K --warmup W --trees B --sims S
                     --root-parallel K --deep --env E --planner P]
"""
import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (ROOT, os.path.join(ROOT, "posggym-baselines_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

# algorithmic HBM bytes (DESIGN.md "Algorithmic bytes"): per simulation, per
# tree level stepped (node 8 + A x 12 child statistics + 84), per leaf expansion
# (A x 20 + 4), per obs node created.  The per-action record is {visits,
# value, total}: ActionNode.agg is not kept, so it is not counted.
# The POMCP search's count is planning/engine.py search_bytes (the same
# constants, and only the work the timed kernel does: no child lookup at a
# deferred level, no child write at a cut-off level, from k_search's
# n_deferred / n_cutoff counters); these are I-NTMCP's (run_intmcp).
B_SIM, B_NEW_NODE = 16, 28
B_LOG_APPEND = 16   # of b_level: the particle-log record (the root level's only HBM term)


def b_level(A):
    return 8 + 12 * A + 84


HBM_PEAK_GBS = 8000.0


def _device_info(dev):
    """Name and compute-unit count of the GPU (the same code measures 3.75-4.73 G
    sims/s across boxes of the pool, DESIGN.md §6: recorded to tell boxes apart)."""
    import torch
    p = torch.cuda.get_device_properties(dev)
    info = {"name": p.name, "gcn_arch": getattr(p, "gcnArchName", ""),
            "compute_units": p.multi_processor_count,
            "hbm_gib": round(p.total_memory / 2**30, 1)}
    if _SMI_STATIC:
        info["smi"] = dict(_SMI_STATIC)
    return info


_SMI_STATIC = {}


def _smi_static():
    """Facts that may differ between boxes (memory vendor, partition modes),
    read from sysfs: no child process is started (under rocprofv3 the GPU is
    initialised before this program runs, and a process that has initialised
    the GPU must not exec another program)."""
    import glob
    for dev in sorted(glob.glob("/sys/class/drm/card*/device")):
        vals = {}
        for key, name in (("GPU memory vendor", "mem_info_vram_vendor"),
                          ("Compute Partition", "current_compute_partition"),
                          ("Memory Partition", "current_memory_partition")):
            try:
                with open(os.path.join(dev, name)) as f:
                    vals[key] = f.read().strip()
            except OSError:
                pass
        if vals:
            _SMI_STATIC.update(vals)
            return


def _lib_sha16():
    """sha256 prefix of the engine library this process loads: PMC traffic in
    profiles/ is reported only when it was measured on this same library."""
    import hashlib
    from posggym_baselines_amd import _native
    with open(_native.LIB_PATH, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()[:16]


def _pmc_traffic(name, lib_sha, **match):
    """HBM bytes per launch from profiles/<name> (tools/summarize_profile.py
    --current) if it was measured on this library and workload, else None."""
    prof = os.path.join(ROOT, "profiles", name)
    try:
        pm = json.load(open(prof))
    except Exception:
        return None
    if pm.get("lib_sha16") != lib_sha:
        return None
    if any(pm.get(k, "Driving-v1" if k == "env" else None) != v for k, v in match.items()):
        return None
    return pm.get("hbm_bytes_per_launch")


def _build_if_missing():
    """The in-tree library is built by __graft_entry__.build() (or here when it
    is missing, before the GPU is touched: hipcc runs as a child process); a
    present library is used as it is -- never rebuilt from inside a profiled
    run."""
    from posggym_baselines_amd import _native
    from posggym_baselines_amd import build as nb
    if not os.path.exists(_native.LIB_PATH):
        nb.build()
    elif not os.environ.get("POMCP_LIB_PATH") and not nb.up_to_date():
        print(f"bench.py: WARNING: {_native.LIB_PATH} is older than its sources (csrc/, "
              "include/); this run measures that library (config.lib_sha16 names it) -- "
              "rebuild with __graft_entry__.build()", file=sys.stderr, flush=True)


class _ClockSampler:
    """Graphics clock and package power read from sysfs (no child process)
    during the timed region, recorded beside the result because the same code
    measures differently on different boxes of the pool.  The
    GPU drawing the most power is reported (this run's, on a one-GPU box).  A
    failure only leaves the list empty."""

    def __init__(self, every_s: float = 0.3):
        import threading
        self.every, self.samples = every_s, []
        self._stop = threading.Event()
        self._t = threading.Thread(target=self._run, daemon=True)

    @staticmethod
    def _read():
        import glob
        best = None
        for dev in glob.glob("/sys/class/drm/card*/device"):
            try:
                with open(os.path.join(dev, "pp_dpm_sclk")) as f:
                    cur = [ln for ln in f.read().splitlines() if ln.strip().endswith("*")]
                sclk = int("".join(ch for ch in cur[0].split(":")[1] if ch.isdigit())) if cur else None
                pw = None
                for h in glob.glob(os.path.join(dev, "hwmon", "hwmon*")):
                    for name in ("power1_average", "power1_input"):
                        fp = os.path.join(h, name)
                        if os.path.exists(fp):
                            with open(fp) as f:
                                pw = int(f.read().strip()) / 1e6
                            break
                    if pw is not None:
                        break
                if best is None or (pw or 0.0) > (best["power_w"] or 0.0):
                    best = {"sclk_mhz": sclk, "power_w": pw}
            except Exception:
                continue
        return best

    def _run(self):
        while not self._stop.is_set() and len(self.samples) < 16:
            r = self._read()
            if r is None:
                return
            self.samples.append(r)
            self._stop.wait(self.every)

    def __enter__(self):
        if not os.environ.get("BENCH_NO_CLOCKS"):
            self._t.start()
        return self

    def __exit__(self, *exc):
        self._stop.set()
        if self._t.is_alive():
            self._t.join(timeout=10)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs = rank processes (default: WORLD_SIZE, else 1); outside a "
                         "torch.distributed launch N > 1 starts the N ranks itself")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--trees", type=int, default=65536)
    ap.add_argument("--sims", type=int, default=None,
                    help="simulations per search (default 65536; intmcp: 256 per nesting level)")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--max-blocks", type=int, default=512,
                    help="per-tree action-block arena; a depth-2 Driving-v1 tree uses ~170 "
                         "(overflow is detected and fails the run)")
    ap.add_argument("--env", default="Driving-v1", choices=["Driving-v1", "PursuitEvasion-v1"],
                    help="Driving-v1 is BASELINE.json's metric; PursuitEvasion-v1 is config 3")
    ap.add_argument("--planner", default="pomcp", choices=["pomcp", "intmcp", "potmmcp"],
                    help="pomcp: BASELINE.json's metric (C2/C3); intmcp: config 5, I-NTMCP "
                         "nesting level 1, one planner pair per lane (--trees pairs, --sims "
                         "simulations per nesting level); potmmcp: POTMMCP with fixed-"
                         "distribution policies (SURVEY §8(f) rank 4), pucb")
    ap.add_argument("--arena", default=None,
                    help="intmcp: per-tree NODES,STATS,LOG arena sizes (skips the calibration "
                         "probe, e.g. for profiling runs)")
    ap.add_argument("--root-parallel", type=int, default=1,
                    help="replica trees per planner: consecutive groups of K trees are one "
                         "planner, merged on the device each step (1 = independent planners)")
    ap.add_argument("--deep", action="store_true",
                    help="gamma=0.99, epsilon=0.01 (depth_limit 459, rollout-dominated)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--update-step", action="store_true",
                    help="each timed step = search + the environment's answer + update() "
                         "(re-root, extraction, reinvigoration, subtree compaction) instead of a "
                         "restore() + search (single GPU)")
    ap.add_argument("--defer", default="auto", choices=["auto", "on", "off"],
                    help="cut-off children deferred to the re-root (pomcp_set_defer_cutoff): "
                         "auto = the planners' default (on)")
    ap.add_argument("--no-sub", action="store_true",
                    help="skip the secondary-configuration records (`sub`) the default run "
                         "appends after the headline (profiling runs)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="collective backend of N > 1 ranks: nccl (= RCCL over xGMI, the "
                         "measurement) or gloo (tests: several ranks sharing one GPU)")
    ap.add_argument("--share-gpu", action="store_true",
                    help="tests only (with --dist-backend gloo): every rank on GPU 0")
    ap.add_argument("--cpu-sample-sims", type=int, default=16384)
    ap.add_argument("--cpu-sample-trees", type=int, default=4)
    ap.add_argument("--cpu-procs", type=int, default=16,
                    help="host processes for the CPU baseline (capped by os.cpu_count(); the "
                         "GPU box's CPU share is 16)")
    args = ap.parse_args()
    if args.sims is None:
        args.sims = 256 if args.planner == "intmcp" else 65536
    if args.trees % args.root_parallel:
        ap.error("--trees must be a multiple of --root-parallel")
    return args


TEST_CFG = dict(discount=0.95, search_time_limit=0.1, c=math.sqrt(2), truncated=False,
                action_selection="ucb", pucb_exploration_fraction=0.25, known_bounds=None,
                step_limit=None, epsilon=0.92, state_belief_only=True)
DEEP_CFG = dict(TEST_CFG, discount=0.99, epsilon=0.01)   # depth_limit 459
# POTMMCP bench: the policy set of tests/golden/potmmcp_pucb.json (three ego
# policies under a meta-policy, a two-policy other-agent mixture)
TM_CFG = dict(TEST_CFG, action_selection="pucb", state_belief_only=False)
TM_SPEC = {"ego": {"u": [0.2] * 5, "acc": [0.1, 0.5, 0.1, 0.2, 0.1],
                   "stay": [0.6, 0.1, 0.1, 0.1, 0.1]},
           "other": {"o_u": [0.2] * 5, "o_fast": [0.05, 0.7, 0.05, 0.1, 0.1]},
           "meta": {"o_u": {"u": 0.5, "acc": 0.25, "stay": 0.25}, "o_fast": {"stay": 0.7, "u": 0.3}}}


def type_policies(model):
    from posggym_baselines_amd.planning import OtherAgentMixturePolicy, POTMMCPMetaPolicy
    from posggym_baselines_amd.planning.policies import FixedDistributionPolicy
    from posggym_baselines_amd.planning.potmmcp import type_policy_tables
    ego = {k: FixedDistributionPolicy(model, "0", k, v) for k, v in TM_SPEC["ego"].items()}
    oth = {k: FixedDistributionPolicy(model, "1", k, v) for k, v in TM_SPEC["other"].items()}
    meta = POTMMCPMetaPolicy(model, "0", ego, TM_SPEC["meta"])
    return type_policy_tables(model, "0", meta, OtherAgentMixturePolicy(model, "1", oth))


def cpu_baseline(sims, trees, seed, env="Driving-v1", first_tree=0, base=None):
    """The oracle (pure-Python restatement of the reference planner, pinned to it by
    tests/golden) timed on one host core over a bounded sample of the same workload."""
    from oracle.episode import run_episode
    from oracle.run import make_oracle
    cfg = dict(base or TEST_CFG, seed=seed)
    t_search = 0.0
    for b in range(first_tree, first_tree + trees):
        p = make_oracle(cfg, sims, tree=b, env=env)

        def step(obs, p=p):
            nonlocal t_search
            p.update(None, obs)
            t0 = time.perf_counter()
            a = p.get_action()
            t_search += time.perf_counter() - t0
            return a

        run_episode(step, 1000 + b, max_steps=1, env=env)
    return {"value": sims * trees / t_search, "unit": "simulations/s", "cores": 1, "kind": "port",
            "sample": f"{trees} roots x {sims} sims (get_action only), oracle/pomcp.py, 1 thread"}


def _cpu_worker(job):
    sims, tree, seed, env, base = job
    r = cpu_baseline(sims, 1, seed, env, first_tree=tree, base=base)
    return sims, sims / r["value"]


def _port_vs_reference():
    """The oracle port's speed relative to the real reference planner on the
    same workload, one core each, as last measured where the reference imports
    (tools/port_vs_reference.py -> profiles/port_vs_reference.json; the
    reference never travels to the GPU box)."""
    try:
        with open(os.path.join(ROOT, "profiles", "port_vs_reference.json")) as f:
            r = json.load(f)
        return {"port_vs_reference_speed": r["port_vs_reference_speed"],
                "port_vs_reference": {k: r[k] for k in ("port_sims_per_s", "reference_sims_per_s",
                                                        "sims", "trees", "cpu", "measured")
                                      if k in r}}
    except (OSError, ValueError, KeyError):
        return {"port_vs_reference_speed": None}


def cpu_baseline_parallel(sims, procs, seed, env="Driving-v1", base=None):
    """The oracle on `procs` host cores at once (one process per core, one root
    each); rate = all simulations / the slowest process's
    search time.  Forked before this process touches the GPU."""
    import multiprocessing as mp
    # close + join (not the context manager, whose exit is terminate(): it
    # SIGTERMs the workers, which a profiler's signal handler reports as an abort)
    pool = mp.get_context("fork").Pool(procs)
    try:
        res = pool.map(_cpu_worker, [(sims, b, seed, env, base) for b in range(procs)])
        pool.close()
    except BaseException:
        pool.terminate()
        raise
    finally:
        pool.join()
    total = sum(r[0] for r in res)
    return {"value": total / max(r[1] for r in res), "unit": "simulations/s", "cores": procs,
            "kind": "port",
            "sample": f"{procs} roots x {sims} sims (get_action only), oracle/pomcp.py, "
                      f"{procs} processes x 1 thread",
            # the port against the real reference planner on the same workload,
            # one core each, measured where the reference imports
            **_port_vs_reference()}


def b_other(A):
    """I-NTMCP level-1 tree level: the other agent's softmax over its level-0
    node (node 8 + A visits x 4) and the level-0 child lookup (16)."""
    return 8 + 4 * A + 16


# per obs node created: its INode (32) + the {obs key, child} slot naming it
# (12; an overflow child's hash entry is 16).  Statistics entries cost no
# bytes inside the search: the node arena is cleared at reset (csrc/intmcp.hip).
B_NODE_IM = 44


def cpu_baseline_intmcp(sims, pairs, seed, env="Driving-v1"):
    """oracle/intmcp.py (pinned to the reference by tests/golden/intmcp_*) timed on
    one host core: get_action of `sims` simulations per level on `pairs` roots."""
    from oracle.episode import run_episode
    from oracle.run import make_oracle_intmcp
    cfg = dict(TEST_CFG, seed=seed, state_belief_only=False)
    t_search = 0.0
    for b in range(pairs):
        p = make_oracle_intmcp(cfg, sims, tree=b, env=env)
        p.reset()

        def step(obs, p=p):
            nonlocal t_search
            top = p.top
            top.update(None, obs)
            t0 = time.perf_counter()
            a = top.get_action(sims)
            t_search += time.perf_counter() - t0
            return a

        run_episode(step, 1000 + b, max_steps=1, env=env)
    return {"value": 2 * sims * pairs / t_search, "unit": "simulations/s", "cores": 1,
            "kind": "port",
            "sample": f"{pairs} roots x {sims} sims per level x 2 levels (get_action only), "
                      "oracle/intmcp.py, 1 thread"}


def run_intmcp(dev, B, S, env, steps, warmup, seed=0, arena=None):
    """I-NTMCP nesting level 1 (BASELINE config 5): B planner pairs x S
    simulations per level, one batched k_im_search launch per step.  Returns
    the bench fields (value, ms_per_step, roofline, config)."""
    import torch
    from posggym_baselines_amd.envs import DrivingModel, PursuitEvasionModel
    from posggym_baselines_amd.planning import BatchedINTMCP, MCTSConfig
    from posggym_baselines_amd.planning.intmcp import plan_intmcp_capacities
    lib_sha = _lib_sha16()
    cfg = MCTSConfig(seed=seed, num_sims=S, **dict(TEST_CFG, state_belief_only=False))
    model = PursuitEvasionModel() if env == "PursuitEvasion-v1" else DrivingModel()
    A = model.action_spaces["0"].n
    searches = warmup + steps + 1
    caps = plan_intmcp_capacities(cfg, model.spec.max_episode_steps, S, searches, A)
    if arena:
        nodes, nstats, nlog = (int(x) for x in arena.split(","))
        caps.max_nodes, caps.max_stats, caps.max_log = nodes, nstats, nlog
        caps.hash_slots = 1 << max(4, (2 * nodes - 1).bit_length())
    elif B > 1024:
        # calibrated arenas: worst-case sizes are ~5x what a search uses; size the
        # per-pair arenas from a 1024-pair probe of the same workload (an overflow
        # would still be detected and fail the run, never be silent)
        probe = BatchedINTMCP(model, "0", cfg, 1024, S, capacities=caps, device=dev)
        probe.init_synthetic(1000 + B)
        for _ in range(searches - 1):
            probe.search(fetch=False)
        ps = probe.engine.root_stats()
        mx = lambda f: max(f(s) for s in ps)
        nodes = int(1.5 * mx(lambda s: max(s.n_nodes[0], s.n_nodes[1]))) + 256
        caps.max_nodes = min(caps.max_nodes, nodes)
        caps.max_log = min(caps.max_log, int(1.5 * mx(lambda s: max(s.n_log[0], s.n_log[1])))
                           + 256)
        caps.max_stats = min(caps.max_stats,
                             int(1.5 * mx(lambda s: max(s.n_stats[0], s.n_stats[1]))) + 64 * A)
        caps.hash_slots = min(caps.hash_slots, 1 << max(4, (2 * nodes - 1).bit_length()))
        probe.close()
    # every timed step searches the same trees again (no restore), so the arenas
    # grow with warmup + steps: say so instead of failing inside hipMalloc
    need, free = caps.bytes_per_pair(A) * B, torch.cuda.mem_get_info(dev)[0]
    if need > 0.95 * free:
        raise SystemExit(f"I-NTMCP arenas for {B} pairs x {searches} searches need "
                         f"{need / 2**30:.0f} GiB, {free / 2**30:.0f} GiB free: "
                         "use fewer --steps/--warmup or --trees")
    stream = torch.cuda.Stream(device=dev)
    bp = BatchedINTMCP(model, "0", cfg, B, S, capacities=caps, stream=stream.cuda_stream,
                       device=dev)
    try:
        bp.init_synthetic(1000)
        for _ in range(warmup):
            with torch.cuda.stream(stream):
                bp.search(fetch=False)
        torch.cuda.synchronize()
        st0 = [(s.n_log[0], s.n_log[1], s.n_nodes[0] + s.n_nodes[1], s.n_stats[0] + s.n_stats[1])
               for s in bp.engine.root_stats()]
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(steps)]
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(steps):
            with torch.cuda.stream(stream):
                ev[k][0].record(stream)
                bp.search(fetch=False)
                ev[k][1].record(stream)
        torch.cuda.synchronize()
        elapsed = time.perf_counter() - t0
        kernel_ms = sum(a.elapsed_time(b) for a, b in ev) / steps
        st = bp.engine.root_stats()
        if any(s.error for s in st):
            raise SystemExit("I-NTMCP search reported an error")
        searched = sum(1 for s in st if not s.root_absorbing)
        lv0 = lv1 = nodes = stats = 0
        for s, s0 in zip(st, st0):
            lv1 += s.n_log[0] - s0[0]
            lv0 += s.n_log[1] - s0[1]
            nodes += s.n_nodes[0] + s.n_nodes[1] - s0[2]
            stats += s.n_stats[0] + s.n_stats[1] - s0[3]
        nodes_used = max(max(s.n_nodes[0], s.n_nodes[1]) for s in st)
    finally:
        bp.close()
    sims_timed = 2 * S * searched * steps
    alg_bytes = (B_SIM * sims_timed + b_level(A) * (lv0 + lv1) + b_other(A) * lv1
                 + B_NODE_IM * nodes) / steps
    achieved = alg_bytes / (kernel_ms * 1e-3) / 1e9
    # the level-1 root's view (node + statistics heads) is served from LDS
    # (ImPair::rv): those bytes of every level-1 simulation's root level never
    # reach HBM
    alg_bytes_hbm = alg_bytes - (8 + 12 * A) * S * searched
    achieved_hbm = alg_bytes_hbm / (kernel_ms * 1e-3) / 1e9
    traffic = _pmc_traffic("pmc_intmcp.json", lib_sha, trees=B, sims=S, env=env)
    return {
        "value": sims_timed / elapsed, "ms_per_step": elapsed * 1e3 / steps,
        "workload": f"I-NTMCP nesting 1 {env}, {B} planner pairs x {S} sims per level x 2 levels "
                    "per step (one batched launch), ucb c=sqrt2 gamma=0.95 depth_limit=2",
        "config": {"pairs": B, "sims_per_level": S, "pairs_searched": searched,
                   "device": _device_info(dev), "lib_sha16": lib_sha,
                   "arena_per_pair": {"max_nodes": caps.max_nodes, "max_stats": caps.max_stats,
                                      "max_log": caps.max_log, "hash_slots": caps.hash_slots,
                                      "bytes": caps.bytes_per_pair(A), "nodes_used": nodes_used}},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "kernel": "k_im_search", "kernel_ms": kernel_ms,
                     "alg_bytes_per_launch": alg_bytes,
                     "alg_bytes_hbm_per_launch": alg_bytes_hbm,
                     "achieved_hbm": achieved_hbm, "frac_hbm": achieved_hbm / HBM_PEAK_GBS},
    }


def main_intmcp(args):
    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1:
        raise SystemExit("--planner intmcp is a single-GPU configuration (BASELINE config 5)")
    _build_if_missing()
    torch.cuda.set_device(0)
    dev = torch.cuda.current_device()
    r = run_intmcp(dev, args.trees, args.sims, args.env, args.steps, args.warmup, args.seed,
                   args.arena)
    out = {
        "metric": f"I-NTMCP simulations/sec on {args.env} (nesting level 1, exact search)",
        "value": r["value"],
        "unit": "simulations/s",
        "n_gpus": 1,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": r["ms_per_step"],
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": f"synthetic {args.env} roots (env seed 1000+b), build's {args.env} restatement",
        "config": dict({"workload": r["workload"]}, **r["config"]),
        "roofline": r["roofline"],
    }
    if not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline_intmcp(2048, 16, args.seed, args.env)
    print(json.dumps(out), flush=True)


def run_pomcp(dev, *, env, B, S, K, base_cfg, tm, steps, warmup, seed=0, max_blocks=512,
              world=1, rank=0, dist=None, update_step=False, clocks=False, defer=None):
    """`steps` timed POMCP steps on B synthetic roots (S simulations each; K
    replica trees per planner, merged on the device).  A step is restore() +
    one k_search launch + the root-parallel exchange, or with `update_step` a
    whole planning step: search, the environment's answer (pomcp_synthetic_step)
    and update() -- re-root, extraction, reinvigoration, subtree compaction --
    before the restore of the next step."""
    import torch
    from posggym_baselines_amd.envs import DrivingModel, PursuitEvasionModel
    from posggym_baselines_amd.planning import BatchedPOMCP, MCTSConfig
    from posggym_baselines_amd.planning.engine import plan_capacities, search_bytes
    from posggym_baselines_amd.planning.parallel import (gather_buffer_tensor, gather_records,
                                                         merge_buffer_tensor)
    lib_sha = _lib_sha16()
    cfg = MCTSConfig(seed=seed, num_sims=S, **base_cfg)
    model = PursuitEvasionModel() if env == "PursuitEvasion-v1" else DrivingModel()
    A = model.action_spaces["0"].n
    step_limit = model.spec.max_episode_steps
    mb = min(max_blocks, S + 64)
    note = ""
    if update_step:
        # the root belief region (pomcp_device.h bel_at) holds the restored root's
        # n_target particles and the re-rooted belief: at most one particle per
        # simulation (a node's records), or 2 n_target while reinvigorating --
        # the worst case, so no probe of the workload is needed
        n_target = cfg.num_particles + cfg.extra_particles
        caps = plan_capacities(cfg, step_limit, S, 1, reroot=True, max_blocks=mb,
                               overflow_slots=1024)
        caps.max_belief = min(caps.max_belief, max(S, 2 * n_target) + n_target + 64)
        free = torch.cuda.mem_get_info(dev)[0]
        while B > 1024 and caps.bytes_per_tree(A, reroot=True) * B > 0.92 * free:
            B //= 2
            note = f" (halved to fit {free / 2**30:.0f} GiB)"
    else:
        caps = plan_capacities(cfg, step_limit, S, 1, reroot=False, max_blocks=mb,
                               overflow_slots=1024)
    stream = torch.cuda.Stream(device=dev)
    # cut-off children deferred to the re-root (the planners' default, the
    # POMCP drop-in's included: pomcp_set_defer_cutoff); defer=False: the eager
    # lookup (a sub record)
    defer = True if defer is None else bool(defer)
    bp = BatchedPOMCP(model, "0", cfg, B, S, capacities=caps, stream=stream.cuda_stream,
                      defer_cutoff=defer,
                      device=dev, type_policies=type_policies(model) if tm else None)
    try:
        bp.init_synthetic(1000)
        bp.engine.rekey(seed ^ (rank << 32))
        merge = merge_buffer_tensor(bp.engine, f"cuda:{dev}")
        gather = gather_buffer_tensor(bp.engine, world, f"cuda:{dev}") if world > 1 else None
        upd_ms = []

        def step(events=None):
            with torch.cuda.stream(stream):
                bp.restore()
                if events is not None:
                    events[0].record(stream)
                if update_step:
                    acts = bp.search(fetch=True)
                else:
                    bp.search(fetch=False)
                if events is not None:
                    events[1].record(stream)
                if update_step:
                    obs = bp.engine.synthetic_step(1000, acts)
                    t1 = time.perf_counter()
                    bp.engine.update(acts, obs)   # synchronises
                    if events is not None:
                        upd_ms.append((time.perf_counter() - t1) * 1e3)
                    return
                # the root-parallel decision: one all-gather of every rank's exchange
                # records (RCCL, same stream), then the device merge of each planner's
                # world x K replicas in replica order (pomcp_merge_roots) -- the same
                # FP64 sums and action on every rank
                if world > 1:   # RCCL: all_gather_into_tensor on this stream (gloo: via host)
                    gather_records(merge, gather)
                bp.engine.merge_roots(K, fetch=False, world=world if world > 1 else 0)

        for _ in range(warmup):
            step()
        torch.cuda.synchronize()
        if not update_step:
            bp.engine.root_stats()   # raises on any per-tree error (arena overflow, ...)
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(steps)]
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        with _ClockSampler() if clocks else _NoClocks() as clk:
            t0 = time.perf_counter()
            for k in range(steps):
                step(ev[k])
            torch.cuda.synchronize()
            if world > 1:
                dist.barrier()
            elapsed = time.perf_counter() - t0
        kernel_ms = sum(a.elapsed_time(b) for a, b in ev) / steps
        if world > 1:
            t = torch.tensor([elapsed, kernel_ms], dtype=torch.float64, device=f"cuda:{dev}")
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            elapsed, kernel_ms = float(t[0]), float(t[1])
        if update_step:   # the search statistics of the last timed step (before its update)
            bp.restore()
            with torch.cuda.stream(stream):
                bp.search(fetch=False)
            torch.cuda.synchronize()
        st = list(bp.engine.root_stats())
        sims = sum(s.num_sims for s in st)          # counted by the kernel, last timed launch
        levels = sum(s.n_levels for s in st)
        deferred = sum(s.n_deferred for s in st)
        cutoff = sum(s.n_cutoff for s in st)
        rollout = sum(s.n_rollout_steps for s in st)
        blocks_used = max(s.n_blocks for s in st)
        log_used = max(s.n_log for s in st)
        if not update_step:
            merged = bp.engine.merge_roots(K, world=world if world > 1 else 0)   # checks errors
            if not all(0 <= m.action < A for m in merged):
                raise SystemExit("merged action out of range")
    finally:
        bp.close()
    # tm: + the action_probs of every stepped node (+ 8A written per leaf expansion)
    alg_bytes = search_bytes(st, A, tm)
    # the root level of every simulation is served from LDS / registers except
    # its particle-log append: its other bytes never reach HBM
    root_levels = min(sims, levels)
    alg_bytes_hbm = alg_bytes - (b_level(A) - B_LOG_APPEND) * root_levels
    achieved = alg_bytes / (kernel_ms * 1e-3) / 1e9
    achieved_hbm = alg_bytes_hbm / (kernel_ms * 1e-3) / 1e9
    counted = sims
    if world > 1:
        t = torch.tensor([counted], dtype=torch.float64, device=f"cuda:{dev}")
        dist.all_reduce(t)   # every rank's counted simulations
        counted = int(t.item())
    # every timed step re-searches the same restored roots: the same count each step
    value = counted * steps / elapsed
    traffic = None if update_step else _pmc_traffic("pmc_search.json", lib_sha, trees=B, sims=S,
                                                     env=env)
    env_desc = ("PursuitEvasion-v1 16x16 max_obs_distance=12" if env == "PursuitEvasion-v1"
                else "Driving-v1 14x14RoundAbout")
    r = {
        "value": value, "ms_per_step": elapsed * 1e3 / steps, "counted": counted,
        "sims_per_step": sims, "B": B, "caps": caps, "clocks": clk.samples, "lib_sha": lib_sha,
        "workload": f"{'POTMMCP' if tm else 'POMCP'} {env_desc} exact search, {B} roots{note} "
                    f"x {S} sims per GPU, {cfg.action_selection} c=sqrt2 "
                    f"gamma={cfg.discount} depth_limit={cfg.depth_limit}, "
                    + ("3 ego policies under a meta-policy, 2 other-agent policies "
                       "(fixed distributions), " if tm else "")
                    + (f"{B // K} planner(s) x {K} replica trees merged on the device, "
                       if K > 1 else "")
                    + ("cut-off children deferred to the re-root, " if defer and not tm else
                       "cut-off children looked up during the search, ")
                    + ("each step = search + env step + update() (re-root, extraction, "
                       "reinvigoration, subtree compaction)" if update_step else
                       f"root-parallel all-gather over {world} GPU(s)"),
        "rollout_steps_per_sim": rollout / max(sims, 1),
        "deferred_levels_per_sim": deferred / max(sims, 1),
        "cutoff_levels_per_sim": cutoff / max(sims, 1), "defer_cutoff": defer,
        "blocks_used": blocks_used, "log_used": log_used, "depth_limit": cfg.depth_limit,
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "kernel": "k_search" if B > 256 or K > 1 else "k_search_lds",
                     "kernel_ms": kernel_ms,
                     "alg_bytes_per_launch": alg_bytes,
                     "alg_bytes_per_sim": alg_bytes / max(sims, 1),
                     # the same without the root level's LDS-served bytes
                     "alg_bytes_hbm_per_launch": alg_bytes_hbm,
                     "achieved_hbm": achieved_hbm, "frac_hbm": achieved_hbm / HBM_PEAK_GBS},
    }
    if update_step:
        r["update_ms"] = sum(upd_ms) / max(1, len(upd_ms))
    return r


class _NoClocks:
    samples = []

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        return False


def _sub(name, r):
    """A compact record of one secondary configuration (the `sub` list)."""
    d = {"name": name, "workload": r["workload"], "value": r["value"], "unit": "simulations/s",
         "ms_per_step": r["ms_per_step"], "kernel": r["roofline"]["kernel"],
         "kernel_ms": r["roofline"]["kernel_ms"], "frac": r["roofline"]["frac"],
         "frac_hbm": r["roofline"]["frac_hbm"]}
    if "defer_cutoff" in r:
        d["defer_cutoff"] = r["defer_cutoff"]
    if "update_ms" in r:
        d["update_ms"] = r["update_ms"]
    return d


def sub_records(dev, seed):
    """BASELINE configs 2 (one root, both single-planner modes), 3 (with the
    update()-inclusive step, so the reinvigoration kernel runs in the timed
    region) and 5, each with a few timed steps; a failure is recorded, never
    fatal to the headline line."""
    jobs = [
        ("C2 headline workload, eager cut-off lookup (pomcp_set_defer_cutoff(0))",
         lambda: run_pomcp(dev, env="Driving-v1", B=65536, S=65536, K=1, base_cfg=TEST_CFG,
                           tm=False, steps=3, warmup=1, seed=seed, defer=False)),
        ("C2 exact single tree (1 x 65536 sims)",
         lambda: run_pomcp(dev, env="Driving-v1", B=1, S=65536, K=1, base_cfg=TEST_CFG, tm=False,
                           steps=3, warmup=1, seed=seed)),
        ("C2 one planner, 1024 replica trees x 64 sims",
         lambda: run_pomcp(dev, env="Driving-v1", B=1024, S=64, K=1024, base_cfg=TEST_CFG,
                           tm=False, steps=20, warmup=5, seed=seed)),
        ("C3 PursuitEvasion-v1 65536 x 65536, update()-inclusive step",
         lambda: run_pomcp(dev, env="PursuitEvasion-v1", B=65536, S=65536, K=1,
                           base_cfg=TEST_CFG, tm=False, steps=2, warmup=1, seed=seed,
                           update_step=True)),
        ("C5 I-NTMCP nesting 1, 65536 pairs x 256 sims per level",
         lambda: run_intmcp(dev, 65536, 256, "Driving-v1", 3, 1, seed)),
    ]
    out = []
    for name, job in jobs:
        t0 = time.perf_counter()
        try:
            d = _sub(name, job())
        except BaseException as e:   # SystemExit included: the headline line still prints
            d = {"name": name, "error": f"{type(e).__name__}: {e}"}
        d["wall_s"] = round(time.perf_counter() - t0, 1)
        out.append(d)
    return out


def _free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_plan(n, argv, port, base_env=None):
    """The N rank processes `python bench.py --gpus N ...` starts when it is not
    already a torch.distributed rank: one process per GPU (the process-per-
    worker shape of baseline_exps/run_planning_exps.py:378-380), each with the
    env torch.distributed.run would give it.  Returns [(argv, env)] by rank."""
    env0 = dict(os.environ if base_env is None else base_env)
    env0.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")   # dmabuf IPC only (RCCL)
    plan = []
    for r in range(n):
        env = dict(env0, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), GROUP_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        plan.append(([sys.executable, "-u", os.path.abspath(__file__)] + list(argv), env))
    return plan


def _gpu_count():
    """Visible GPUs, counted without initialising the GPU in this process
    (torch.cuda.device_count() does not on this image): the launcher starts its
    rank processes afterwards and must never run GPU code itself."""
    import torch
    return torch.cuda.device_count()


def spawn_ranks(n, argv):
    """`--gpus N > 1` outside a torch.distributed launch: check that N GPUs are
    visible, start N rank processes (before this process touches the GPU), wait
    for them and exit with the first failing rank's status (0 if all pass).
    Rank 0 prints the JSON line; a rank that fails ends the others."""
    have = _gpu_count()
    if "--share-gpu" in argv and have >= 1:   # tests: ranks share GPU 0 (gloo)
        have = n
    if have < n:
        print(f"bench.py: --gpus {n} needs {n} visible GPUs, this node has {have}: "
              "nothing was run", file=sys.stderr, flush=True)
        return 3
    import signal
    import subprocess
    plan = launch_plan(n, argv, _free_port())

    def _term(signum, frame):   # the launcher's own SIGTERM ends its ranks (finally below)
        raise SystemExit(128 + signum)
    signal.signal(signal.SIGTERM, _term)
    procs = [subprocess.Popen(a, env=e) for a, e in plan]
    rc = 0
    try:
        live = list(procs)
        while live:
            for p in list(live):
                r = p.poll()
                if r is None:
                    continue
                live.remove(p)
                if r != 0 and rc == 0:
                    rc = r if r > 0 else 128 - r
                    print(f"bench.py: rank {procs.index(p)} exited with {r}; stopping the "
                          "other ranks", file=sys.stderr, flush=True)
                    for q in live:
                        q.send_signal(signal.SIGTERM)
            time.sleep(0.2)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
            p.wait()
    return rc


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "0") or 0)
    if world == 0 and (args.gpus or 1) > 1:
        # not a torch.distributed rank: become the launcher of N ranks (no GPU
        # work in this process, so no exec-after-GPU-init hazard)
        if args.planner == "intmcp":
            raise SystemExit("--planner intmcp is a single-GPU configuration (BASELINE config 5)")
        sys.exit(spawn_ranks(args.gpus, sys.argv[1:]))
    world = world or 1
    if args.gpus is None:
        args.gpus = world
    if args.gpus != world:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}: launch one "
                         "process per GPU (torch.distributed.run --nproc-per-node N ... "
                         "--gpus N, or python bench.py --gpus N)")
    _smi_static()   # before anything touches the GPU
    if args.planner == "intmcp":
        return main_intmcp(args)
    import torch
    import torch.distributed as dist

    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    cpu = None
    base_cfg = DEEP_CFG if args.deep else TEST_CFG
    tm = args.planner == "potmmcp"
    if tm:
        if args.env != "Driving-v1" or args.deep:
            raise SystemExit("--planner potmmcp: Driving-v1, default configuration")
        base_cfg = TM_CFG
    # (no CPU leg for POTMMCP: the oracle has no restatement of it -- its parity
    # is pinned to the reference's own records)
    if rank == 0 and not args.no_cpu_baseline and not tm:
        # before any GPU call: the worker processes are forked from this one.
        # With N ranks rank 0 runs it before the process group forms (the other
        # ranks wait in its rendezvous), so every line carries its CPU baseline;
        # the timed steps start after run_pomcp's barrier, so it is never in the
        # measured time
        procs = max(1, min(args.cpu_procs, os.cpu_count() or 1))
        sample = args.cpu_sample_sims if not args.deep else max(64, args.cpu_sample_sims // 8)
        cpu = cpu_baseline_parallel(sample, procs, args.seed, args.env, base_cfg)
    if rank == 0:
        _build_if_missing()
    rccl_ranks = None
    if world > 1:
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        if args.share_gpu:
            if args.dist_backend != "gloo":
                raise SystemExit("bench.py: --share-gpu needs --dist-backend gloo")
            local = 0
        if local >= torch.cuda.device_count():
            raise SystemExit(f"bench.py: rank {rank} (LOCAL_RANK {local}) has no GPU: "
                             f"{torch.cuda.device_count()} visible")
        torch.cuda.set_device(local)
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")
        formed = dist.get_world_size()
        if formed != world:
            raise SystemExit(f"bench.py: the process group formed with {formed} ranks, "
                             f"expected {world}")
        rccl_ranks = formed if args.dist_backend == "nccl" else None
    else:
        torch.cuda.set_device(0)
    dev = torch.cuda.current_device()
    if world > 1:
        dist.barrier()   # rank 0's build is complete
    B, S, K = args.trees, args.sims, args.root_parallel
    if args.update_step and (world > 1 or K > 1):
        raise SystemExit("--update-step: one GPU, independent planners")
    r = run_pomcp(dev, env=args.env, B=B, S=S, K=K, base_cfg=base_cfg, tm=tm, steps=args.steps,
                  warmup=args.warmup, seed=args.seed, max_blocks=args.max_blocks, world=world,
                  rank=rank, dist=dist if world > 1 else None, clocks=True,
                  update_step=args.update_step,
                  defer=None if args.defer == "auto" else args.defer == "on")
    caps = r["caps"]
    out = {
        "metric": (f"MCTS simulations/sec on {args.env} (POTMMCP exact search, fixed-distribution "
                   "policies)" if tm else f"MCTS simulations/sec on {args.env} (POMCP exact search)"),
        "value": r["value"],
        "unit": "simulations/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": r["ms_per_step"],
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": f"synthetic {args.env} belief states (env seed 1000+b), build's {args.env} "
                "restatement",
        "config": {"workload": r["workload"],
                   "trees_per_gpu": r["B"], "sims_per_tree": S, "depth_limit": r["depth_limit"],
                   "root_parallel": K, "planners_per_gpu": r["B"] // K,
                   "sims_per_planner_step": S * K,
                   "rollout_steps_per_sim": r["rollout_steps_per_sim"],
                   "deferred_levels_per_sim": r["deferred_levels_per_sim"],
                   "cutoff_levels_per_sim": r["cutoff_levels_per_sim"],
                   "defer_cutoff": r["defer_cutoff"],
                   "collective": (args.dist_backend if world > 1 else None),
                   "parallelism": f"root-parallel x{world}",
                   "rccl_ranks": rccl_ranks,
                   "device": dict(_device_info(dev), during_run=r["clocks"]),
                   "lib_sha16": r["lib_sha"], "counted_sims_per_step": r["counted"],
                   "arena": {"max_blocks": caps.max_blocks,
                             "max_blocks_used": r["blocks_used"],
                             "max_particles": caps.max_particles,
                             "max_particles_used": r["log_used"]}},
        "roofline": r["roofline"],
    }
    if "update_ms" in r:
        out["update_ms"] = r["update_ms"]
    if cpu is not None:
        out["cpu_baseline"] = cpu
    default_run = (world == 1 and not tm and not args.deep and args.env == "Driving-v1"
                   and B == 65536 and S == 65536 and K == 1 and not args.update_step)
    if rank == 0 and default_run and not args.no_sub:
        out["sub"] = sub_records(dev, args.seed)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
