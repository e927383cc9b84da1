"""Drop-in for ``posggym_baselines.planning`` (``planning/__init__.py:1-18``):
the POMCP / I-NTMCP hot path on MI355X."""
from posggym_baselines_amd.planning.config import MCTSConfig  # noqa: F401
from posggym_baselines_amd.planning.episodes import (  # noqa: F401
    EpisodeResultsWriter,
    run_planning_episodes,
)
from posggym_baselines_amd.planning.intmcp import INTMCP, BatchedINTMCP  # noqa: F401
from posggym_baselines_amd.planning.ipomcp import IPOMCP, MCTS  # noqa: F401
from posggym_baselines_amd.planning.other_policy import (  # noqa: F401
    OtherAgentMixturePolicy,
    OtherAgentPolicy,
    RandomOtherAgentPolicy,
)
from posggym_baselines_amd.planning.pomcp import POMCP, BatchedPOMCP, uct_merge  # noqa: F401
from posggym_baselines_amd.planning.potmmcp import POTMMCP, POTMMCPMetaPolicy  # noqa: F401
from posggym_baselines_amd.planning.search_policy import (  # noqa: F401
    PPOLSTMSearchPolicy,
    RandomSearchPolicy,
    SearchPolicy,
    SearchPolicyWrapper,
    load_posggym_agents_search_policy,
)
from posggym_baselines_amd.planning.utils import (  # noqa: F401
    KnownBounds,
    MinMaxStats,
    PlanningStatTracker,
)
