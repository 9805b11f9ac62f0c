"""Index sharding of environments over the GPUs of one node.

Envs are independent, so rank ``r`` of ``W`` simply owns a contiguous slice of the global
env index range.  Everything random is a pure function of the global index, so a sharded
rollout is bit-identical to the single-GPU one:

* reset keys:  ``split(key, B_total + 1)[1 + lo : 1 + hi]``  (VmapGymWrapper reset closure,
  wrappers.py:160-164) -- computed per rank with ``pob_random_split(first=1 + lo)``;
* actions:     ``uniform(split(key)[1], (B_total, A), -1, 1)[lo:hi]``  (pob_random_actions).

No collective is on the data path; ``gather_obs`` (RCCL all-gather over xGMI) assembles
the final observation batch on every rank when a learner needs it.
"""
from __future__ import annotations

from typing import Tuple


def shard_range(total: int, world: int, rank: int) -> Tuple[int, int]:
    """[lo, hi) of the global env indices owned by ``rank`` (balanced, contiguous)."""
    if world <= 0 or not (0 <= rank < world):
        raise ValueError("bad world/rank")
    base, rem = divmod(total, world)
    lo = rank * base + min(rank, rem)
    hi = lo + base + (1 if rank < rem else 0)
    return lo, hi


def shard_keys(key, total: int, world: int, rank: int):
    """This rank's reset keys: rows [1 + lo, 1 + hi) of split(key, total + 1) (device)."""
    import torch
    from . import _lib
    from ._lib import lib, check
    lo, hi = shard_range(total, world, rank)
    out = torch.empty((hi - lo, 2), dtype=torch.uint32, device=key.device)
    if hi > lo:
        check(lib.pob_random_split(key.data_ptr(), total + 1, 1 + lo, hi - lo, out.data_ptr(),
                                   _lib.stream_handle(key.device)))
    return out


def gather_obs(obs, group=None):
    """All-gather the (B_local, D) observation shards of every rank -> (B_total, D).

    torch.distributed with the "nccl" backend is RCCL on ROCm (xGMI within a node).
    Equal shard sizes are required (use a total divisible by the world size)."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    out = torch.empty((world * obs.shape[0],) + tuple(obs.shape[1:]), dtype=obs.dtype, device=obs.device)
    dist.all_gather_into_tensor(out, obs.contiguous(), group=group)
    return out
