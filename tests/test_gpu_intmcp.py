"""GPU parity of the I-NTMCP engine (BASELINE config 5) through the C ABI:
every step record of the reference goldens (level-1 root statistics, root
particles with the other agent's histories, every level-0 node those histories
name: visits, children, particles) must match bit for bit."""
import pytest

from golden_util import INTMCP_CASES, cfg_kwargs, load
from gpu_util import gpu_intmcp_episode

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("case", INTMCP_CASES)
def test_gpu_intmcp_matches_reference_goldens(case):
    data = load(case)
    for ep in data["episodes"]:
        kw = cfg_kwargs(ep["config"])
        trace, records = gpu_intmcp_episode(kw, data["num_sims"], ep["env_seed"],
                                            ego=data["ego"], max_steps=data["max_steps"],
                                            env=data["env"])
        assert len(records) == len(ep["records"]), case
        for t, (got, exp) in enumerate(zip(records, ep["records"])):
            assert got == exp, f"{case} env_seed {ep['env_seed']} step {t}"
        assert trace == ep["trace"]
