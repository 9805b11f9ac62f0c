"""Index sharding of environments over the GPUs of one node.

Envs are independent, so rank ``r`` of ``W`` simply owns a contiguous slice of the global
env index range.  Everything random is a pure function of the global index, so a sharded
rollout is bit-identical to the single-GPU one:

* reset keys:  ``split(key, B_total + 1)[1 + lo : 1 + hi]``  (VmapGymWrapper reset closure,
  wrappers.py:160-164) -- computed per rank with ``pob_random_split(first=1 + lo)``;
* actions:     ``uniform(split(key)[1], (B_total, A), -1, 1)[lo:hi]``  (pob_random_actions);
* gym autoreset (``AutoresetVmapGymWrapper.step``, wrappers.py:245-262): the reference
  advances ONE gym key whenever ANY env of the whole batch is done.  Sharded, each rank's
  step kernel sets a local any-done word, ``all_reduce_any_done`` takes the MAX over
  ranks (one 4-byte RCCL all-reduce per step, stream-ordered, no host sync), and the
  masked reset draws rank-local rows ``split(gym_key, B_total + 1)[1 + lo + b]``
  (``pob_reset_where_done_shard``).

The plain brax path has no collective on the data path; ``gather_obs`` (RCCL all-gather
over xGMI) assembles the observation batch on every rank when a learner needs it.  The
helpers work with any torch.distributed backend ("nccl" = RCCL on ROCm; "gloo" on CPU
tensors in the tests).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Any, Optional, Tuple


def shard_range(total: int, world: int, rank: int) -> Tuple[int, int]:
    """[lo, hi) of the global env indices owned by ``rank`` (balanced, contiguous)."""
    if world <= 0 or not (0 <= rank < world):
        raise ValueError("bad world/rank")
    base, rem = divmod(total, world)
    lo = rank * base + min(rank, rem)
    hi = lo + base + (1 if rank < rem else 0)
    return lo, hi


@dataclass(frozen=True)
class Shard:
    """This process's slice of a global env batch (``total`` envs over ``world`` ranks)."""
    total: int
    world: int = 1
    rank: int = 0
    group: Any = None

    def __post_init__(self):
        if self.total <= 0:
            raise ValueError("total batch must be positive")
        shard_range(self.total, self.world, self.rank)  # validates world / rank

    @property
    def lo(self) -> int:
        return shard_range(self.total, self.world, self.rank)[0]

    @property
    def hi(self) -> int:
        return shard_range(self.total, self.world, self.rank)[1]

    @property
    def size(self) -> int:
        lo, hi = shard_range(self.total, self.world, self.rank)
        return hi - lo

    def gym_key_rows(self) -> Tuple[int, int, int]:
        """(num, first, count) of this rank's rows of split(gym_key, total + 1)."""
        return self.total + 1, 1 + self.lo, self.size

    @classmethod
    def current(cls, total: int, group=None) -> "Shard":
        """The shard of this process under torch.distributed (world 1 when not initialised)."""
        import torch.distributed as dist
        if dist.is_available() and dist.is_initialized():
            return cls(total, dist.get_world_size(group), dist.get_rank(group), group)
        return cls(total)


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


def all_reduce_any_done(flag, group=None):
    """In place: this rank's any-done word (``flag[0]``, uint32 0/1, written by the step
    kernel) becomes the MAX over all ranks.  A no-op outside torch.distributed; with a process
    group it runs at any world size, 1 included (the one-GPU box exercises it over RCCL).
    4 bytes per call; on RCCL it is stream-ordered (no host sync)."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return flag
    v = flag[:1].view(torch.int32) if flag.dtype == torch.uint32 else flag[:1]
    dist.all_reduce(v, op=dist.ReduceOp.MAX, group=group)
    return flag


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


def gather_obs_ragged(obs, total: int, group=None):
    """gather_obs for unequal shards (shard_range of ``total``): every rank's rows padded to
    the largest shard, gathered, and the padding dropped -> (total, D)."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    m = max(hi - lo for lo, hi in (shard_range(total, world, r) for r in range(world)))
    pad = torch.zeros((m,) + tuple(obs.shape[1:]), dtype=obs.dtype, device=obs.device)
    pad[:obs.shape[0]] = obs
    full = gather_obs(pad, group)
    return torch.cat([full[r * m: r * m + (hi - lo)]
                      for r, (lo, hi) in enumerate(shard_range(total, world, r) for r in range(world))])


class ObsGatherer:
    """Double-buffered all-gather of each step's observation batch, overlapped with the
    following steps ("overlap it with the next step via a separate stream").

    ``submit(obs)`` is called on the compute stream right after step t's kernel: it copies
    this rank's obs rows into staging slot ``p = t % depth`` (one D2D copy on the compute
    stream, so step t + 1 may overwrite ``obs`` at once) and enqueues the all-gather of that
    slot into ``full[p]`` on a side stream, ordered after the copy by an event.  Step t + 1's
    kernel therefore runs concurrently with step t's gather; slot ``p`` is reused by step
    t + depth, whose copy waits (on the device, not the host) for gather t to finish.
    ``result(p)`` makes the caller's current stream wait for gather ``p`` and returns the
    (B_total, D) batch in global env order; it stays valid until ``depth`` more submits.

    Unequal shards (``shard_range`` of ``total``) are padded to the largest shard and the
    padding is dropped by ``result``.  On CPU tensors (gloo) the same rotation runs
    synchronously, which is what the world-2 tests exercise."""

    def __init__(self, total: int, D: int, dtype=None, device=None, group=None, depth: int = 2):
        import torch
        import torch.distributed as dist
        self.total, self.D, self.group = int(total), int(D), group
        # (with a process group the all-gather runs at any world size, 1 included: the one-GPU
        # box exercises RCCL and the side-stream ordering through it)
        self.dist = dist.is_available() and dist.is_initialized()
        self.world = dist.get_world_size(group) if self.dist else 1
        self.rank = dist.get_rank(group) if self.dist else 0
        self.bounds = [shard_range(self.total, self.world, r) for r in range(self.world)]
        self.m = max(hi - lo for lo, hi in self.bounds)
        self.ragged = any(hi - lo != self.m for lo, hi in self.bounds)
        self.depth = max(1, int(depth))
        dtype = dtype or torch.float32
        self.device = torch.device(device) if device is not None else torch.device("cpu")
        self.cuda = self.device.type == "cuda"
        self.stage = [torch.zeros((self.m, self.D), dtype=dtype, device=self.device) for _ in range(self.depth)]
        self.full = [torch.empty((self.world * self.m, self.D), dtype=dtype, device=self.device)
                     for _ in range(self.depth)]
        self.stream = torch.cuda.Stream(self.device) if self.cuda else None
        self._done = [None] * self.depth    # event: gather of slot p finished (side stream)
        self._t0 = [None] * self.depth      # event: gather of slot p enqueued (timing)
        self.k = 0

    def submit(self, obs) -> int:
        """Stage ``obs`` (this rank's (B_local, D) rows) and start its all-gather; returns
        the slot to pass to ``result``."""
        import torch
        import torch.distributed as dist
        lo, hi = self.bounds[self.rank]
        if tuple(obs.shape) != (hi - lo, self.D):
            raise ValueError(f"obs shard {tuple(obs.shape)} != ({hi - lo}, {self.D})")
        p = self.k % self.depth
        self.k += 1
        if not self.cuda:
            self.stage[p][:hi - lo].copy_(obs)
            if self.dist:
                dist.all_gather_into_tensor(self.full[p], self.stage[p], group=self.group)
            else:
                self.full[p].copy_(self.stage[p])
            return p
        cur = torch.cuda.current_stream(self.device)
        if self._done[p] is not None:
            cur.wait_event(self._done[p])  # gather t - depth has read the slot
        self.stage[p][:hi - lo].copy_(obs)
        staged = torch.cuda.Event()
        staged.record(cur)
        with torch.cuda.stream(self.stream):
            self.stream.wait_event(staged)
            t0 = torch.cuda.Event(enable_timing=True)
            t0.record(self.stream)
            if self.dist:
                dist.all_gather_into_tensor(self.full[p], self.stage[p], group=self.group)
            else:
                self.full[p].copy_(self.stage[p])
            done = torch.cuda.Event(enable_timing=True)
            done.record(self.stream)
        self._t0[p], self._done[p] = t0, done
        return p

    def result(self, p: int):
        """The gathered (B_total, D) observation batch of slot ``p`` (global env order)."""
        import torch
        if self.cuda and self._done[p] is not None:
            torch.cuda.current_stream(self.device).wait_event(self._done[p])
        f = self.full[p]
        if not self.ragged:
            return f
        return torch.cat([f[r * self.m: r * self.m + (hi - lo)] for r, (lo, hi) in enumerate(self.bounds)])

    def gather_ms(self, p: int) -> float:
        """Device time of slot p's last gather (side stream, from its start to its end)."""
        return self._t0[p].elapsed_time(self._done[p]) if self.cuda and self._done[p] is not None else 0.0
