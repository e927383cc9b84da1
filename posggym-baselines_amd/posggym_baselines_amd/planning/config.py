"""``MCTSConfig`` — same fields, checks and derived values as the reference's
``posggym_baselines/planning/config.py:8-55``, plus two engine fields.

Additive fields (defaults keep the reference behaviour):
  * ``num_sims``: run exactly this many simulations per ``get_action`` instead
    of the wall-clock loop of ``mcts.py:285`` (needed for reproducible parity);
  * ``device``: HIP device ordinal of the engine;
  * ``root_parallel``: K replica trees for one planner on the GPU (replica k =
    the exact planner with RNG key (seed, k); ``num_sims`` is split as
    ceil(num_sims / K) per replica; the final action is the device merge of the
    replicas' root statistics, ``pomcp_merge_roots``).  1 (default) = the
    reference's single tree, bit-exact.
"""
import math
from dataclasses import dataclass, field
from typing import Optional

from posggym_baselines_amd.planning.utils import KnownBounds


@dataclass
class MCTSConfig:
    discount: float
    search_time_limit: float
    c: float
    truncated: bool
    action_selection: str = "pucb"
    pucb_exploration_fraction: float = 0.5
    known_bounds: Optional[KnownBounds] = None
    extra_particles_prop: float = 1.0 / 16
    reinvigoration_sample_limit_factor: float = 4.0
    step_limit: Optional[int] = None
    epsilon: float = 0.01
    seed: Optional[int] = None
    state_belief_only: bool = False
    use_rollout_if_no_value: bool = True
    num_sims: Optional[int] = None
    device: int = 0
    root_parallel: int = 1

    num_particles: int = field(init=False)
    extra_particles: int = field(init=False)
    depth_limit: int = field(init=False)

    def __post_init__(self):
        # same assertions (AssertionError) as config.py:34-45
        assert 0.0 <= self.discount <= 1.0
        assert self.search_time_limit > 0.0
        assert self.c > 0.0
        assert 0.0 <= self.pucb_exploration_fraction <= 1.0
        assert 0.0 <= self.extra_particles_prop <= 1.0
        assert 0.0 < self.epsilon < 1.0
        self.action_selection = self.action_selection.lower()
        assert self.action_selection in ("pucb", "ucb", "uniform")
        assert self.num_sims is None or self.num_sims >= 0
        assert self.root_parallel >= 1
        # derived sizes, config.py:47-55 (discount == 1 raises ZeroDivisionError there too)
        self.num_particles = math.ceil(self.search_time_limit * 100)
        self.extra_particles = math.ceil(self.extra_particles_prop * self.num_particles)
        self.depth_limit = 0 if self.discount == 0.0 else math.ceil(
            math.log(self.epsilon) / math.log(self.discount))
