"""ctypes binding of libpomcp_hip.so (include/pomcp.h).

The structs below mirror the C declarations field for field.  The library is
built in-tree by ``posggym_baselines_amd.build`` (hipcc, gfx950) and loaded
from ``posggym_baselines_amd/_lib/``; there is no fallback: if the shared
object is missing, importing the planner raises.
"""
import ctypes as C
import os

LIB_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_lib")
LIB_PATH = os.environ.get("POMCP_LIB_PATH") or os.path.join(LIB_DIR, "libpomcp_hip.so")

POMCP_ABI_VERSION = 7
POMCP_MAX_TYPE_POLICIES = 8
POMCP_MAX_ACTIONS = 8
POMCP_XREC_STATS = 6


def xrec(num_actions: int) -> int:
    """Doubles per tree in the exchange record (include/pomcp.h POMCP_XREC)."""
    return 2 * num_actions + POMCP_XREC_STATS

POMCP_OK = 0
POMCP_E_INVALID = -1
POMCP_E_HIP = -2
POMCP_E_ARENA = -3
POMCP_E_STATE = -4
POMCP_E_UNSUPPORTED = -5
POMCP_E_NOT_FOUND = -6
POMCP_E_NO_DEVICE = -7

SEL_PUCB, SEL_UCB, SEL_UNIFORM = 0, 1, 2
SEARCH_AUTO, SEARCH_LANE, SEARCH_WAVE = 0, 1, 2   # pomcp_search_kernel
ENV_DRIVING = 1
ENV_PURSUIT_EVASION = 2

STATUS_NAMES = {
    POMCP_E_INVALID: "POMCP_E_INVALID",
    POMCP_E_HIP: "POMCP_E_HIP",
    POMCP_E_ARENA: "POMCP_E_ARENA",
    POMCP_E_STATE: "POMCP_E_STATE",
    POMCP_E_UNSUPPORTED: "POMCP_E_UNSUPPORTED",
    POMCP_E_NOT_FOUND: "POMCP_E_NOT_FOUND",
    POMCP_E_NO_DEVICE: "POMCP_E_NO_DEVICE",
}


class PomcpGrid(C.Structure):
    _fields_ = [
        ("wall", C.c_uint8 * 256),
        ("dist", (C.c_uint8 * 256) * 8),
        ("loc_x", C.c_uint8 * 8),
        ("loc_y", C.c_uint8 * 8),
        ("loc_dir", C.c_uint8 * 8),
        ("width", C.c_int32),
        ("height", C.c_int32),
        ("num_locs", C.c_int32),
        ("obs_front", C.c_int32),
        ("obs_back", C.c_int32),
        ("obs_side", C.c_int32),
        ("pad", C.c_int32 * 2),
    ]


class PomcpPeGrid(C.Structure):
    _fields_ = [
        ("wall", C.c_uint8 * 256),
        ("goal_dist", (C.c_uint8 * 256) * 4),
        ("evader_start", (C.c_uint8 * 2) * 4),
        ("pursuer_start", (C.c_uint8 * 2) * 4),
        ("goal", (C.c_uint8 * 2) * 4),
        ("width", C.c_int32),
        ("height", C.c_int32),
        ("n_evader_start", C.c_int32),
        ("n_pursuer_start", C.c_int32),
        ("n_goal", C.c_int32),
        ("max_obs_distance", C.c_int32),
        ("use_progress_reward", C.c_int32),
        ("pad", C.c_int32),
        ("reward_norm", C.c_double),
    ]


class PomcpConfig(C.Structure):
    _fields_ = [
        ("abi_version", C.c_int32),
        ("env_id", C.c_int32),
        ("num_agents", C.c_int32),
        ("ego_agent", C.c_int32),
        ("num_actions", C.c_int32),
        ("action_selection", C.c_int32),
        ("depth_limit", C.c_int32),
        ("step_limit", C.c_int32),
        ("num_particles", C.c_int32),
        ("extra_particles", C.c_int32),
        ("has_known_bounds", C.c_int32),
        ("num_trees", C.c_int32),
        ("discount", C.c_double),
        ("c", C.c_double),
        ("pucb_exploration_fraction", C.c_double),
        ("reinvigoration_sample_limit_factor", C.c_double),
        ("known_min", C.c_double),
        ("known_max", C.c_double),
        ("seed", C.c_uint64),
        ("tree_key_base", C.c_uint32),
        ("type_based", C.c_int32),
        ("max_blocks", C.c_int64),
        ("max_particles", C.c_int64),
        ("max_belief", C.c_int64),
        ("overflow_slots", C.c_int64),
        ("log_table", C.POINTER(C.c_double)),
        ("log_table_size", C.c_int64),
        ("discount_pow", C.POINTER(C.c_double)),
        ("discount_pow_size", C.c_int64),
        ("grid", PomcpGrid),
        ("pe_grid", PomcpPeGrid),
    ]


class PomcpRootStats(C.Structure):
    _fields_ = [
        ("action", C.c_int32),
        ("num_sims", C.c_int32),
        ("search_depth", C.c_int32),
        ("root_visits", C.c_int32),
        ("root_absorbing", C.c_int32),
        ("belief_size", C.c_int32),
        ("error", C.c_int32),
        ("num_children", C.c_int32),
        ("child_visits", C.c_int32 * POMCP_MAX_ACTIONS),
        ("child_values", C.c_double * POMCP_MAX_ACTIONS),
        ("child_totals", C.c_double * POMCP_MAX_ACTIONS),
        ("min_value", C.c_double),
        ("max_value", C.c_double),
        ("n_levels", C.c_int64),
        ("n_expansions", C.c_int64),
        ("n_new_nodes", C.c_int64),
        ("n_rollout_steps", C.c_int64),
        ("n_probes", C.c_int64),
        ("n_obs_nodes", C.c_int32),
        ("n_blocks", C.c_int32),
        ("n_log", C.c_int32),
        ("n_deferred", C.c_int32),
        ("n_cutoff", C.c_int32),
        ("n_exact_selects", C.c_int32),
    ]


class PomcpMergedRoot(C.Structure):
    """``pomcp_merged_root`` (include/pomcp.h)."""
    _fields_ = [
        ("action", C.c_int32),
        ("num_trees", C.c_int32),
        ("search_depth", C.c_int32),
        ("error", C.c_int32),
        ("num_sims", C.c_int64),
        ("root_visits", C.c_int64),
        ("min_value", C.c_double),
        ("max_value", C.c_double),
        ("visits", C.c_double * POMCP_MAX_ACTIONS),
        ("totals", C.c_double * POMCP_MAX_ACTIONS),
    ]


# (name, restype, argtypes) for every symbol include/pomcp.h declares.
_CTX = C.c_void_p
class PomcpTypePolicies(C.Structure):
    """``pomcp_type_policies`` (include/pomcp.h): POTMMCP's fixed-distribution policies."""
    _fields_ = [
        ("num_ego", C.c_int32),
        ("num_other", C.c_int32),
        ("ego_pi", (C.c_double * POMCP_MAX_ACTIONS) * POMCP_MAX_TYPE_POLICIES),
        ("other_pi", (C.c_double * POMCP_MAX_ACTIONS) * POMCP_MAX_TYPE_POLICIES),
        ("meta_len", C.c_int32 * POMCP_MAX_TYPE_POLICIES),
        ("meta_policy", (C.c_int32 * POMCP_MAX_TYPE_POLICIES) * POMCP_MAX_TYPE_POLICIES),
        ("meta_weight", (C.c_double * POMCP_MAX_TYPE_POLICIES) * POMCP_MAX_TYPE_POLICIES),
        ("expected_prior", C.c_double * POMCP_MAX_ACTIONS),
        ("no_meta_draw", C.c_int32),
        ("no_mixture_draw", C.c_int32),
        ("ego_uniform", C.c_int32),
        ("other_uniform", C.c_int32),
    ]


_P32 = C.POINTER(C.c_int32)
_PU32 = C.POINTER(C.c_uint32)
_PU64 = C.POINTER(C.c_uint64)
_PD = C.POINTER(C.c_double)
SIGNATURES = [
    ("pomcp_abi_version", C.c_int32, []),
    ("pomcp_create", C.c_int, [C.POINTER(PomcpConfig), C.c_int32, C.c_void_p, C.POINTER(_CTX)]),
    ("pomcp_destroy", None, [_CTX]),
    ("pomcp_last_error", C.c_char_p, [_CTX]),
    ("pomcp_set_stream", C.c_int, [_CTX, C.c_void_p]),
    ("pomcp_reset", C.c_int, [_CTX]),
    ("pomcp_update", C.c_int, [_CTX, _P32, _PU64, _P32]),
    ("pomcp_search", C.c_int, [_CTX, C.c_int32, _P32]),
    ("pomcp_search_continue", C.c_int, [_CTX, C.c_int32]),
    ("pomcp_set_search_kernel", C.c_int, [_CTX, C.c_int32]),
    ("pomcp_search_kernel_used", C.c_int32, [_CTX]),
    ("pomcp_set_defer_cutoff", C.c_int, [_CTX, C.c_int32]),
    ("pomcp_get_root_stats", C.c_int, [_CTX, C.POINTER(PomcpRootStats)]),
    ("pomcp_set_root_belief", C.c_int, [_CTX, C.c_int32, _PU32, C.c_int32]),
    ("pomcp_get_root_belief", C.c_int, [_CTX, C.c_int32, _PU32, C.c_int32, _P32]),
    ("pomcp_set_type_policies", C.c_int, [_CTX, C.POINTER(PomcpTypePolicies)]),
    ("pomcp_get_root_prior", C.c_int, [_CTX, C.c_int32, _PD]),
    ("pomcp_get_root_policies", C.c_int, [_CTX, C.c_int32, _P32, C.c_int32, _P32]),
    ("pomcp_arena_usage", C.c_int, [_CTX, _P32, _P32]),
    ("pomcp_rekey", C.c_int, [_CTX, C.c_uint64]),
    ("pomcp_root_merge_buffer", C.c_int, [_CTX, C.POINTER(C.c_void_p)]),
    ("pomcp_root_gather_buffer", C.c_int, [_CTX, C.c_int32, C.POINTER(C.c_void_p)]),
    ("pomcp_allgather_root", C.c_int, [_CTX, C.c_void_p, C.c_int32]),
    ("pomcp_merge_roots", C.c_int, [_CTX, C.c_int32, C.c_int32, C.POINTER(PomcpMergedRoot)]),
    ("pomcp_synthetic_obs", C.c_int, [_CTX, C.c_uint64, _PU64]),
    ("pomcp_synthetic_step", C.c_int, [_CTX, C.c_uint64, _P32, _PU64]),
    ("pomcp_snapshot", C.c_int, [_CTX]),
    ("pomcp_restore", C.c_int, [_CTX]),
    ("pomcp_driving_sample_initial_state", C.c_int,
     [C.POINTER(PomcpGrid), C.c_uint64, C.c_uint32, _PU32, _PU32]),
    ("pomcp_driving_step", C.c_int,
     [C.POINTER(PomcpGrid), C.c_uint64, C.c_uint32, _PU32, _PU32, _P32, _PU32, _PD, _P32, _PU64]),
    ("pomcp_driving_obs", C.c_int, [C.POINTER(PomcpGrid), _PU32, _PU64]),
    ("pomcp_pe_sample_initial_state", C.c_int,
     [C.POINTER(PomcpPeGrid), C.c_uint64, C.c_uint32, _PU32, _PU32]),
    ("pomcp_pe_step", C.c_int, [C.POINTER(PomcpPeGrid), _PU32, _P32, _PU32, _PD, _P32, _PU64]),
    ("pomcp_pe_obs", C.c_int, [C.POINTER(PomcpPeGrid), _PU32, _PU64]),
    ("pomcp_philox_words", C.c_int, [C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32, C.c_int32,
                                     _PU32]),
    ("pomcp_host_log_table", C.c_int, [C.c_int64, C.c_int64, _PD]),
]
DEBUG_SIGNATURES = [
    ("pomcp_debug_fp_selftest", C.c_int, [_PD, _PD, C.c_int32, _PD]),
    ("pomcp_debug_exp", C.c_int, [_PD, C.c_int32, _PD]),
    ("pomcp_debug_fast_recip", C.c_int, [_PD, C.c_int32, _PD]),
    ("pomcp_debug_host_exp", C.c_int, [_PD, C.c_int32, _PD]),
    ("pomcp_debug_phase_timing", C.c_int,
     [C.c_void_p, C.POINTER(C.c_uint64), C.c_int32, C.POINTER(C.c_int32)]),
    ("pomcp_debug_set_inline_slots", C.c_int, [C.c_void_p, C.c_int32]),
    ("pomcp_debug_set_select_margin", C.c_int, [C.c_void_p, C.c_double]),
    ("pomcp_debug_set_spin_limit", C.c_int, [C.c_void_p, C.c_int32]),
    ("intmcp_debug_set_softmax_slack", C.c_int, [C.c_void_p, C.c_float]),
    ("intmcp_debug_exact_draws", C.c_int, [C.c_void_p, C.POINTER(C.c_uint64)]),
]



class IntmcpConfig(C.Structure):
    """``intmcp_config`` (include/intmcp.h)."""
    _fields_ = [
        ("base", PomcpConfig),
        ("state_belief_only", C.c_int32),
        ("nesting_level", C.c_int32),
        ("max_nodes", C.c_int64),
        ("max_stats", C.c_int64),
        ("max_log", C.c_int64),
        ("hash_slots", C.c_int64),
        ("max_root_belief", C.c_int64),
        ("max_support_particles", C.c_int64),
    ]


class IntmcpRootStats(C.Structure):
    """``intmcp_root_stats`` (include/intmcp.h)."""
    _fields_ = [
        ("action", C.c_int32),
        ("num_sims", C.c_int32),
        ("search_depth", C.c_int32),
        ("root_visits", C.c_int32),
        ("root_absorbing", C.c_int32),
        ("belief_size", C.c_int32),
        ("error", C.c_int32),
        ("num_children", C.c_int32),
        ("child_action", C.c_int32 * POMCP_MAX_ACTIONS),
        ("child_visits", C.c_int32 * POMCP_MAX_ACTIONS),
        ("child_values", C.c_double * POMCP_MAX_ACTIONS),
        ("child_totals", C.c_double * POMCP_MAX_ACTIONS),
        ("min_value", C.c_double),
        ("max_value", C.c_double),
        ("n_nodes", C.c_int32 * 2),
        ("n_log", C.c_int32 * 2),
        ("n_stats", C.c_int32 * 2),
        ("n_support", C.c_int32),
        ("pad", C.c_int32),
    ]


INTMCP_BEGIN, INTMCP_FINAL = 1, 2
INTMCP_SKIP = -2

# numpy views of the diagnostic records (include/intmcp.h)
INTMCP_NODE_DTYPE = [("parent", "<i4"), ("info", "<u4"), ("visits", "<i4"), ("t", "<i4"),
                     ("stats", "<i4"), ("support", "<u4"), ("okey", "<u8")]
INTMCP_STAT_DTYPE = [("visits", "<i4"), ("pad", "<i4"), ("value", "<f8"), ("total", "<f8"),
                     ("agg", "<f8")]
INTMCP_SUPPORT_DTYPE = [("node", "<i4"), ("off", "<i4"), ("size", "<i4"), ("cap", "<i4")]

INTMCP_SIGNATURES = [
    ("intmcp_create", C.c_int, [C.POINTER(IntmcpConfig), C.c_int32, C.c_void_p, C.POINTER(_CTX)]),
    ("intmcp_destroy", None, [_CTX]),
    ("intmcp_last_error", C.c_char_p, [_CTX]),
    ("intmcp_reset", C.c_int, [_CTX]),
    ("intmcp_update", C.c_int, [_CTX, _P32, _PU64, _P32]),
    ("intmcp_search", C.c_int, [_CTX, C.c_int32, _P32]),
    ("intmcp_search_levels", C.c_int, [_CTX, C.c_int32, C.c_int32, C.c_int32, _P32]),
    ("intmcp_get_root_stats", C.c_int, [_CTX, C.POINTER(IntmcpRootStats)]),
    ("intmcp_get_root_belief", C.c_int, [_CTX, C.c_int32, _PU32, C.c_int32, _P32]),
    ("intmcp_get_nodes", C.c_int, [_CTX, C.c_int32, C.c_int32, C.c_void_p, C.c_int32, _P32]),
    ("intmcp_get_stats", C.c_int, [_CTX, C.c_int32, C.c_int32, C.c_void_p, C.c_int32, _P32]),
    ("intmcp_get_support", C.c_int,
     [_CTX, C.c_int32, _P32, C.c_int32, _P32, _PU32, C.c_int32, _P32]),
    ("intmcp_get_mid_support", C.c_int,
     [_CTX, C.c_int32, _P32, C.c_int32, _P32, _PU32, C.c_int32, _P32]),
    ("intmcp_get_middle_support", C.c_int,
     [_CTX, C.c_int32, C.c_int32, _P32, C.c_int32, _P32, _PU32, C.c_int32, _P32]),
    ("intmcp_search_level", C.c_int, [_CTX, C.c_int32, C.c_int32, C.c_int32, _P32]),
    ("intmcp_get_tree_counts", C.c_int, [_CTX, _P32]),
    ("intmcp_synthetic_obs", C.c_int, [_CTX, C.c_uint64, _PU64]),
    ("intmcp_set_search_policy", C.c_int, [_CTX, C.c_int32, C.c_int32, _PD]),
    ("intmcp_debug_phase_timing", C.c_int, [_CTX, C.c_void_p, C.c_int32, _P32]),
]

_lib = None


class PomcpError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"{STATUS_NAMES.get(code, code)}: {msg}")
        self.code = code


def load():
    """Load the in-tree shared object (raises if it was never built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} is missing: build it with `python -m posggym_baselines_amd.build` "
            "(or __graft_entry__.build()); there is no CPU fallback for the planner")
    # One HIP runtime per process: PyTorch ships its own libamdhip64.so.7 (same
    # soname as /opt/rocm's).  Whichever loads first serves both; torch only
    # initialises on its own copy, so it is loaded before this library.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = C.CDLL(LIB_PATH)
    for name, res, args in SIGNATURES + DEBUG_SIGNATURES + INTMCP_SIGNATURES:
        if (name, res, args) in DEBUG_SIGNATURES and not hasattr(lib, name):
            continue   # diagnostics: optional in libraries built from older sources
        if os.environ.get("POMCP_LIB_PATH") and not hasattr(lib, name):
            continue   # an explicitly chosen (measurement) library built from older sources
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.pomcp_abi_version() != POMCP_ABI_VERSION:
        raise ImportError("libpomcp_hip.so ABI version mismatch; rebuild")
    _lib = lib
    return lib


def check(rc, ctx=None, what="", last_error="pomcp_last_error"):
    if rc != POMCP_OK:
        msg = what
        if ctx is not None:
            err = getattr(load(), last_error)(ctx)
            if err:
                msg = f"{what}: {err.decode()}"
        raise PomcpError(rc, msg)
