from posggym_baselines_amd.envs.driving import (  # noqa: F401
    GRIDS,
    DrivingModel,
    pack_obs,
    unpack_obs,
)
from posggym_baselines_amd.envs.pursuit_evasion import PursuitEvasionModel  # noqa: F401
