"""Root-parallel search across GPUs.

Every rank searches the same roots with its own RNG key; at action-selection
time one all-reduce (RCCL over xGMI for backend "nccl", gloo in CPU tests)
sums each root action's (visit count, total value) and every rank takes the
same merged decision: argmax of total / visits, lowest action on ties
(the merged form of ``max_value_action_selection``, mcts.py:583-600).
"""
import math

import torch
import torch.distributed as dist


class _DeviceArray:
    """``__cuda_array_interface__`` view of a device pointer owned by the engine."""

    def __init__(self, ptr, n):
        self.__cuda_array_interface__ = {"shape": (n,), "typestr": "<f8", "data": (ptr, False),
                                         "version": 3}


def merge_buffer_tensor(engine, device):
    """The engine's ``double[trees][A][2]`` merge buffer as a torch tensor (no copy)."""
    n = engine.num_trees * engine.A * 2
    return torch.as_tensor(_DeviceArray(engine.merge_buffer_ptr(), n), device=device)


def root_parallel_merge(merge: torch.Tensor, num_actions: int, world_size: int = 1):
    """All-reduce (visits, total) per root action and return the merged actions."""
    if world_size > 1:
        dist.all_reduce(merge)
    m = merge.view(-1, num_actions, 2)
    vis, tot = m[..., 0], m[..., 1]
    val = torch.where(vis > 0, tot / vis.clamp_min(1), torch.full_like(tot, -math.inf))
    return torch.argmax(val, dim=-1)
