"""Root-parallel merge and root-parallel planner — CPU restatement.

TEST INFRASTRUCTURE (see ``oracle/__init__.py``).

The reference has no root-parallel planner: every ``MCTS`` searches one tree
and ends ``get_action`` with ``_final_action_selection`` (``mcts.py:565-600``).
The build's root-parallel mode (``MCTSConfig.root_parallel``)
runs K replica trees of one planner -- replica k is exactly the oracle planner
with RNG key (seed, k) -- and replaces the final selection by a merge of the
replicas' root statistics.  This module restates that merge
(``k_merge_roots``, csrc/pomcp_kernels.hip) in the same summation order, and
drives K oracle planners through an episode the way the drop-in does.
"""
import math

INF = float("inf")


def merge_roots(visits, totals, sel):
    """Merge N replicas' root children: ``visits[j][a]``, ``totals[j][a]``.

    Across ranks (``pomcp_merge_roots`` after the all-gather) replica j = r * K
    + k is replica k of rank r, so the list is rank-major.
    Fixed summation order: lane l of 64 sums replicas [l*c, (l+1)*c), c =
    ceil(N / 64), in order from 0.0; the 64 partials are summed in lane order
    from 0.0.  PUCB: argmax of summed visits (``max_visit_action_selection``,
    ``mcts.py:565-581``); UCB / uniform: argmax of summed total / summed visits
    over visited actions (``max_value_action_selection``, ``mcts.py:583-600``);
    lowest action on ties; 0 when nothing was visited (``mcts.py:270-272``).
    Returns (action, summed visits, summed totals)."""
    K = len(visits)
    A = len(visits[0]) if K else 0
    c = (K + 63) // 64
    pv = [[0.0] * A for _ in range(64)]
    pt = [[0.0] * A for _ in range(64)]
    for lane in range(64):
        for k in range(min(lane * c, K), min(lane * c + c, K)):
            for a in range(A):
                pv[lane][a] = pv[lane][a] + float(visits[k][a])
                pt[lane][a] = pt[lane][a] + float(totals[k][a])
    sv, st = [0.0] * A, [0.0] * A
    for lane in range(64):
        for a in range(A):
            sv[a] = sv[a] + pv[lane][a]
            st[a] = st[a] + pt[lane][a]
    action, best, found = 0, 0.0, False
    for a in range(A):
        if not sv[a] > 0.0:
            continue
        score = sv[a] if sel == "pucb" else st[a] / sv[a]
        if not found or score > best:
            action, best, found = a, score, True
    return action, sv, st


class OracleRootParallel:
    """K oracle planners (keys (seed, 0..K-1)) driven as one root-parallel
    planner: every replica is updated with the merged action and the real
    observation, searches ``ceil(num_sims / K)`` simulations, and the merged
    action is played."""

    def __init__(self, planners, sel):
        self.planners = planners
        self.sel = sel
        self.last_action = None
        self.merged = None

    def absorbing(self):
        """The planner is absorbing when every replica's root is (a replica
        whose root is absorbing does not search and merges as zeros)."""
        return all(p.on_abs[p.root] for p in self.planners)

    def step(self, obs):
        ps = self.planners
        if self.absorbing():
            return self.last_action
        for p in ps:
            p.stats = {"searched": True}
            p.update(self.last_action, obs)
        if self.absorbing():
            self.merged = None
            self.last_action = 0                      # mcts.py:270-272
            return self.last_action
        for p in ps:
            p.get_action()
        zeros = [0] * ps[0].A
        self.merged = merge_roots([p.stats.get("child_visits", zeros) for p in ps],
                                  [p.stats.get("child_totals", zeros) for p in ps], self.sel)
        self.last_action = self.merged[0]
        return self.last_action


def per_replica_sims(num_sims, K):
    return math.ceil(num_sims / K)
