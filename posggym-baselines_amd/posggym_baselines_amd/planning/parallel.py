"""Root-parallel search across GPUs.

Every rank searches the same roots with its own RNG keys; at action-selection
time ONE all-reduce (RCCL over xGMI for backend "nccl", gloo in CPU tests) sums
each root action's (visit count, total value) in the engine's merge buffer, and
every rank takes the same merged decision on the device
(``PomcpEngine.merge_roots`` / ``pomcp_merge_roots``):

* PUCB: argmax of summed visits (the merged ``max_visit_action_selection``,
  ``mcts.py:565-581``);
* UCB / uniform: argmax of summed total / summed visits over visited actions
  (the merged ``max_value_action_selection``, ``mcts.py:583-600``);

lowest action on ties.  RCCL's ring all-reduce leaves bit-identical sums on
every rank, so every rank plays the same action.
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


def allreduce_roots(engine, device, group=None):
    """Sum the merge buffer over the ranks of ``group`` in place (one collective).

    The engine's kernels run on its own HIP stream while torch.distributed
    enqueues on torch's current stream, so the two are ordered by host
    synchronisation: ``root_stats``/``search(fetch=True)`` have synchronised
    the engine before, and the caller's ``merge_roots`` (engine stream) follows
    ``torch.cuda.synchronize``."""
    buf = merge_buffer_tensor(engine, device)
    dist.all_reduce(buf, group=group)
    if buf.is_cuda:
        torch.cuda.synchronize(buf.device)
    return buf


def root_parallel_merge(merge: torch.Tensor, num_actions: int, world_size: int = 1,
                        action_selection: str = "ucb"):
    """All-reduce (visits, total) per root action and return the merged actions
    (torch restatement of the decision rule, for host tensors; the GPU path
    uses the device merge ``PomcpEngine.merge_roots``)."""
    if world_size > 1:
        dist.all_reduce(merge)
    m = merge.view(-1, num_actions, 2)
    vis, tot = m[..., 0], m[..., 1]
    if action_selection == "pucb":
        score = torch.where(vis > 0, vis, torch.full_like(vis, -math.inf))
    else:
        score = torch.where(vis > 0, tot / vis.clamp_min(1), torch.full_like(tot, -math.inf))
    # lowest action on ties: first index of the maximum; 0 if nothing was visited
    best = score.max(dim=-1, keepdim=True).values
    first = (score == best) & (vis > 0)
    idx = torch.arange(num_actions, device=merge.device).expand_as(first)
    act = torch.where(first, idx, torch.full_like(idx, num_actions)).min(dim=-1).values
    return torch.where(act == num_actions, torch.zeros_like(act), act)
