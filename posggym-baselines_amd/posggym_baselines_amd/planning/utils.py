"""Host-side planning utilities: ``KnownBounds``, ``MinMaxStats`` and the
per-step statistics contract ``PlanningStatTracker``
(``posggym_baselines/planning/utils.py:12-144``).  On the GPU the min/max
statistics live in two registers per tree; this class is for host code that
wants the same normalisation."""
from collections import namedtuple
from typing import Dict, List, Optional

import numpy as np

KnownBounds = namedtuple("KnownBounds", ["min", "max"])


class MinMaxStats:
    """Running tree-wide value bounds (MuZero pseudocode; utils.py:15-42)."""

    def __init__(self, known_bounds: Optional[KnownBounds]):
        if known_bounds:
            self.minimum, self.maximum = known_bounds.min, known_bounds.max
        else:
            self.minimum, self.maximum = float("inf"), -float("inf")

    def update(self, value: float):
        if value > self.maximum:
            self.maximum = value
        if value < self.minimum:
            self.minimum = value

    def normalize(self, value: float) -> float:
        if self.maximum > self.minimum:
            return (value - self.minimum) / (self.maximum - self.minimum)
        return value

    def __str__(self):
        return f"MinMaxState: (minimum: {self.minimum}, maximum: {self.maximum})"


class PlanningStatTracker:
    """Per-step / per-episode aggregation of ``planner.step_statistics``.

    Same keys and reductions as utils.py:45-144: mean per episode except
    ``mem_usage`` (max); NaN steps (absorbing root) are skipped by the nan-
    reductions.
    """

    STAT_KEYS = ["search_time", "update_time", "reinvigoration_time", "evaluation_time",
                 "policy_calls", "inference_time", "search_depth", "num_sims", "mem_usage",
                 "min_value", "max_value"]
    MAX_STATS = {"mem_usage"}

    def __init__(self, planner, track_overall: bool = True):
        self.planner = planner
        self.track_overall = track_overall
        self.reset()

    def _empty(self) -> Dict[str, List[float]]:
        return {k: [] for k in self.STAT_KEYS}

    def step(self):
        self._current_steps += 1
        for k in self.STAT_KEYS:
            self._current_stats[k].append(self.planner.step_statistics.get(k, np.nan))

    def reset(self):
        self._current_steps = 0
        self._current_stats = self._empty()
        self._num_episodes = 0
        self._all_steps: List[int] = []
        self._all_stats = self._empty()

    def reset_episode(self):
        if self._current_steps == 0:
            return
        self._num_episodes += 1
        if self.track_overall:
            self._all_steps.append(self._current_steps)
            for k in self.STAT_KEYS:
                red = np.nanmax if k in self.MAX_STATS else np.nanmean
                self._all_stats[k].append(red(self._current_stats[k]))
        self._current_steps = 0
        self._current_stats = self._empty()

    def get_episode(self) -> Dict[str, float]:
        out = {}
        for k, vals in self._current_stats.items():
            if len(vals) == 0 or np.isnan(np.sum(vals)):
                out[k] = np.nan
            else:
                out[k] = (np.nanmax if k in self.MAX_STATS else np.nanmean)(vals, axis=0)
        return out

    def get(self) -> Dict[str, float]:
        out = {}
        for k, vals in self._all_stats.items():
            if len(vals) == 0 or np.isnan(np.sum(vals)):
                out[f"{k}_mean"] = out[f"{k}_std"] = np.nan
                continue
            out[f"{k}_mean"] = (np.nanmax if k in self.MAX_STATS else np.nanmean)(vals, axis=0)
            out[f"{k}_std"] = np.nanstd(vals, axis=0)
        return out
