"""Environment registry of the oracle (TEST INFRASTRUCTURE, see ``oracle/__init__.py``).

The two generative models the GPU engine implements, each the build's
restatement of a posggym environment (parity with posggym unpinned)."""
from oracle.driving import DrivingModel
from oracle.pursuit_evasion import PursuitEvasionModel

DEFAULT_GRID = {"Driving-v1": "14x14RoundAbout", "PursuitEvasion-v1": "16x16"}


def make_model(env, streams, grid=None):
    grid = grid or DEFAULT_GRID[env]
    if env == "Driving-v1":
        return DrivingModel(streams, grid=grid)
    if env == "PursuitEvasion-v1":
        return PursuitEvasionModel(streams, grid=grid)
    raise KeyError(env)
