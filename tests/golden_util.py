"""Helpers to load the committed golden fixtures (tests/golden/*.json)."""
import json
import os

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
EPISODE_CASES = ["c1_ucb", "c1_pucb", "uniform", "deep_ucb", "known_bounds", "ego1_ucb",
                 "large_first_step"]


def load(name):
    with open(os.path.join(GOLDEN, f"{name}.json")) as f:
        return json.load(f)


def cfg_kwargs(cfg):
    kw = dict(cfg)
    if kw.get("known_bounds") is not None:
        kw["known_bounds"] = tuple(kw["known_bounds"])
    return kw
