"""Root-parallel search across GPUs.

Every rank searches the same roots with its own RNG keys.  At action-selection
time ONE all-gather (RCCL over xGMI for backend "nccl"; gloo in CPU tests)
collects every rank's exchange records -- per tree the (visit count, total
value) of each root action and the search's step statistics, include/pomcp.h
``POMCP_XREC`` -- into the engine's gather buffer in rank order, and every
rank takes the same merged decision on the device (``PomcpEngine.merge_roots``
/ ``pomcp_merge_roots`` with ``world`` ranks):

* PUCB: argmax of summed visits (the merged ``max_visit_action_selection``,
  ``mcts.py:565-581``);
* UCB / uniform: argmax of summed total / summed visits over visited actions
  (the merged ``max_value_action_selection``, ``mcts.py:583-600``);

lowest action on ties.  The merge sums the world x K replica records in one
fixed order (replica j = rank * K + k), so the FP64 sums -- and the action --
are the same on every rank, whatever the number of ranks and whatever
algorithm the collective library picks, and equal a single GPU merging all
world x K replicas (restated by ``oracle/root_parallel.py``).  An all-reduce
would leave the summation order to RCCL (ring chunks rotate it per rank
count), which no restatement can follow beyond two ranks.
"""
import numpy as np
import torch
import torch.distributed as dist

from posggym_baselines_amd._native import xrec


class _DeviceArray:
    """``__cuda_array_interface__`` view of a device pointer owned by the engine."""

    def __init__(self, ptr, n):
        self.__cuda_array_interface__ = {"shape": (n,), "typestr": "<f8", "data": (ptr, False),
                                         "version": 3}


def merge_buffer_tensor(engine, device):
    """The engine's ``double[trees][xrec(A)]`` exchange records as a torch tensor
    (no copy)."""
    n = engine.num_trees * xrec(engine.A)
    return torch.as_tensor(_DeviceArray(engine.merge_buffer_ptr(), n), device=device)


def gather_buffer_tensor(engine, world, device):
    """The engine's ``double[world][trees][xrec(A)]`` gather buffer (no copy)."""
    n = world * engine.num_trees * xrec(engine.A)
    return torch.as_tensor(_DeviceArray(engine.gather_buffer_ptr(world), n), device=device)


def gather_records(local: torch.Tensor, out: torch.Tensor, group=None):
    """All-gather every rank's records ``local`` into ``out`` (``world *
    local.numel()``, rank order).  RCCL gathers device tensors directly on
    torch's current stream; other backends (gloo) stage through host memory."""
    world = dist.get_world_size(group)
    if out.numel() != world * local.numel():
        raise ValueError("gather buffer size != world x records")
    if dist.get_backend(group) == "nccl":
        dist.all_gather_into_tensor(out, local, group=group)
        return out
    host = local.detach().to("cpu")
    parts = [torch.empty_like(host) for _ in range(world)]
    dist.all_gather(parts, host, group=group)
    out.copy_(torch.cat(parts).to(out.device))
    return out


def exchange_roots(engine, device, group=None):
    """The root-parallel exchange: all-gather of the engine's records into its
    gather buffer; returns the world size to pass to ``engine.merge_roots``.

    The engine's kernels run on its own HIP stream while torch.distributed
    enqueues on torch's current stream, so the two are ordered by host
    synchronisation: the device is synchronised before the gather (the search
    has written the records) and after it (the merge, on the engine's stream,
    reads the gather buffer)."""
    world = dist.get_world_size(group)
    local = merge_buffer_tensor(engine, device)
    out = gather_buffer_tensor(engine, world, device)
    if local.is_cuda:
        torch.cuda.synchronize(local.device)
    gather_records(local, out, group)
    if out.is_cuda:
        torch.cuda.synchronize(out.device)
    return world


def allgather_small(values, group=None, device=None):
    """All-gather a few float64 per rank (flags, counters) -> numpy [world, n].
    One tiny collective; device tensors for RCCL, host tensors otherwise."""
    world = dist.get_world_size(group)
    v = torch.tensor([float(x) for x in values], dtype=torch.float64)
    if dist.get_backend(group) == "nccl":
        v = v.to(device if device is not None else "cuda")
        out = torch.empty(world * v.numel(), dtype=torch.float64, device=v.device)
        dist.all_gather_into_tensor(out, v, group=group)
        return out.cpu().numpy().reshape(world, -1)
    parts = [torch.empty_like(v) for _ in range(world)]
    dist.all_gather(parts, v, group=group)
    return torch.stack(parts).numpy()


class PeerFailure(RuntimeError):
    """Raised on the ranks whose own step succeeded when a peer rank's failed:
    every rank leaves the collective sequence together instead of waiting
    forever for the failed one."""


def raise_together(exc, row_values, group=None, device=None):
    """Agree on failure before the data collective: every rank contributes
    (failed, *row_values); if any rank failed, all raise (the failing rank its
    own exception).  Returns the gathered [world, 1 + n] rows otherwise."""
    rows = allgather_small([1.0 if exc is not None else 0.0] + list(row_values), group, device)
    if exc is not None:
        raise exc
    bad = np.nonzero(rows[:, 0])[0]
    if len(bad):
        raise PeerFailure(f"root-parallel peer rank(s) {bad.tolist()} failed")
    return rows
