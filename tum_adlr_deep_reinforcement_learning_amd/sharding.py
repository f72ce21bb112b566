"""Env sharding across the GPUs of a node.

Aircraft are independent, so a global batch of envs splits into contiguous
ranges, one per process/GPU, with no collective on the env-step path.  Rank r's
engine seeds its Philox streams with ``env_offset`` = the first global env id
it owns, which makes every trajectory independent of the sharding (tested
bitwise).  The two real exchanges -- the end-of-collection rollout all-gather
and the per-step VecNormalize moment records -- go through
:func:`all_gather_flat`: one ``all_gather_into_tensor`` on RCCL (``nccl``), a
list ``all_gather`` on ``gloo`` (CPU tests).
"""
import os

import torch
import torch.distributed as dist


def world():
    """(rank, world_size, local_rank) from torchrun's environment (1 process = rank 0 of 1)."""
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size(), int(os.environ.get("LOCAL_RANK", "0"))
    return int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("LOCAL_RANK", "0"))


def shard_range(n_total, rank, world_size):
    """Contiguous split of ``n_total`` envs: (env_offset, count) of ``rank`` (first ranks get the remainder).

    An uneven split is fine for stepping; the rollout all-gather needs equal shards and raises on one
    (RolloutBuffer.all_gather)."""
    base, rem = divmod(int(n_total), int(world_size))
    count = base + (1 if rank < rem else 0)
    offset = rank * base + min(rank, rem)
    return offset, count


def all_gather_flat(t, group=None, out=None):
    """Gather a contiguous tensor from every rank -> [W][t.numel()] (rank order).

    Without a process group this is a view of ``t``.  With one (any size, also world 1) it is a real
    collective: ``all_gather_into_tensor`` on RCCL (``nccl``), a list ``all_gather`` on gloo.  ``out``
    (optional, [W * t.numel()] of t's dtype/device) receives the result in place, so a caller can keep
    the destination at a fixed address (a captured graph reads it)."""
    t = t.contiguous().view(-1)
    if not (dist.is_available() and dist.is_initialized()):
        if out is not None:
            out.view(-1).copy_(t)
            return out.view(1, -1)
        return t.view(1, -1)
    W = dist.get_world_size(group)
    if out is None:
        out = torch.empty(W * t.numel(), dtype=t.dtype, device=t.device)
    elif out.numel() != W * t.numel() or out.dtype != t.dtype or out.device != t.device:
        raise ValueError("all_gather_flat: out must hold world_size * t.numel() elements of t's dtype and device")
    if dist.get_backend(group) == "nccl":
        dist.all_gather_into_tensor(out, t, group=group)
    else:
        dist.all_gather(list(out.view(W, -1)), t, group=group)
    return out.view(W, -1)
