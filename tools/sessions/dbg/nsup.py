import os, sys, collections
ROOT = "/root/repo"
sys.path[:0] = [ROOT, os.path.join(ROOT, "posggym-baselines_amd")]
import torch
torch.cuda.init()
from bench import TEST_CFG
from posggym_baselines_amd.envs import DrivingModel
from posggym_baselines_amd.planning import BatchedINTMCP, MCTSConfig
cfg = MCTSConfig(seed=1, num_sims=256, **dict(TEST_CFG, state_belief_only=False))
bp = BatchedINTMCP(DrivingModel(), "0", cfg, 4096, 256, searches=3)
bp.init_synthetic(1000)
st = bp.engine.root_stats()
print("n_support", sorted(collections.Counter(s.n_support for s in st).items()))
print("belief", sorted(collections.Counter(s.belief_size for s in st).items())[:10])
bp.close()
