"""CPU, world_size 2 (gloo): index sharding of envs reproduces the single-process batch.

Each rank takes its slice of split(key, B+1)[1:] (po_brax_amd.sharding.shard_range), runs
the CPU oracle's reset + steps on it with its slice of the global action batch, and the
all-gathered shards must equal the unsharded run bit for bit -- the property the GPU
bench relies on.
"""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

B, T = 48, 3


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(rank, world, port, name, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "po-brax_amd"), os.path.join(root, "oracle")]
    import orc
    import pob_np as P
    from po_brax_amd.sharding import shard_range
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lo, hi = shard_range(B, world, rank)
    key = P.prngkey(0)
    keys = P.split(key, B + 1)[1 + lo:1 + hi]
    e = orc.OracleEnv(name)
    s = e.reset(keys, first=True)
    for t in range(T):
        key, k = P.split(key)
        act = P.uniform(k, (B, 8), -1, 1)[lo:hi]
        s = e.step(s, act, flags=orc.F_EPISODE | orc.F_AUTORESET, episode_length=2)
    obs = torch.from_numpy(s["obs"])
    parts = [torch.empty_like(obs) for _ in range(world)]
    dist.all_gather(parts, obs)
    if rank == 0:
        q.put(torch.cat(parts).numpy())
    dist.destroy_process_group()


def _single(name):
    import orc
    import pob_np as P
    key = P.prngkey(0)
    e = orc.OracleEnv(name)
    s = e.reset(P.split(key, B + 1)[1:], first=True)
    for t in range(T):
        key, k = P.split(key)
        s = e.step(s, P.uniform(k, (B, 8), -1, 1), flags=orc.F_EPISODE | orc.F_AUTORESET, episode_length=2)
    return s["obs"]


def test_sharded_equals_single_world2():
    ctx = mp.get_context("spawn")
    for name in ("ant_heavenhell", "ant_tag"):
        q = ctx.Queue()
        port = _free_port()
        procs = [ctx.Process(target=_run, args=(r, 2, port, name, q)) for r in range(2)]
        for p in procs:
            p.start()
        got = q.get(timeout=120)
        for p in procs:
            p.join(timeout=120)
            assert p.exitcode == 0
        np.testing.assert_array_equal(got, _single(name))


def test_shard_range_covers():
    from po_brax_amd.sharding import shard_range
    for total in (1, 7, 64, 65536, 262144):
        for world in (1, 2, 3, 8):
            rs = [shard_range(total, world, r) for r in range(world)]
            assert rs[0][0] == 0 and rs[-1][1] == total
            assert all(a[1] == b[0] for a, b in zip(rs, rs[1:]))


# ---------------------------------------------------------------- sharded gym autoreset
BG, TG, LG = 49, 9, 4  # ragged shards (25 + 24), episodes of 4 steps -> several gym resets


def _gym_rank(rank, world, port, name, q, force=None):
    """One rank of a sharded AutoresetVmapGymWrapper loop, with the PRODUCT's host logic
    (po_brax_amd.sharding: Shard rows of the global gym-key split, the any-done all-reduce,
    the ragged obs all-gather) and the CPU oracle as the per-env compute (the GPU box runs
    the same logic over RCCL with the HIP kernels, pob_reset_where_done_shard)."""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "po-brax_amd"), os.path.join(root, "oracle")]
    import orc
    import pob_np as P
    from po_brax_amd.sharding import Shard, all_reduce_any_done, gather_obs_ragged
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sh = Shard.current(BG)
    assert (sh.world, sh.rank) == (world, rank)
    num, first, count = sh.gym_key_rows()
    gkey = P.prngkey(3)
    ks = P.split(gkey, num)
    e = orc.OracleEnv(name)
    s = e.reset(ks[first:first + count])
    gkey = ks[0].copy()
    akey = P.prngkey(8)
    any_steps = 0
    split_flags = []  # (step, local any-done, global any-done) where they differ
    for t in range(TG):
        akey, k = P.split(akey)
        act = P.uniform(k, (BG, 8), -1, 1)[sh.lo:sh.hi]
        s = e.step(s, act, flags=orc.F_EPISODE, episode_length=LG)
        if force is not None and t == force[0] and sh.lo <= force[1] < sh.hi:
            s["done"][force[1] - sh.lo] = 1.0  # one env of one rank ends its episode early
        local = 1 if (s["done"] != 0).any() else 0
        flag = torch.tensor([local, 0, 0, 0], dtype=torch.uint32)
        all_reduce_any_done(flag)
        if local != int(flag[0]):
            split_flags.append((t, local, int(flag[0])))
        if int(flag[0]):  # wrappers.py:247-261 on this rank's rows of the global split
            any_steps += 1
            ks = P.split(gkey, num)
            gkey = ks[0].copy()
            d = s["done"] != 0
            if d.any():
                fresh = e.reset(ks[first:first + count][d])
                for f in ("pos", "rot", "vel", "ang", "obs"):
                    s[f][d] = fresh[f]
                s["steps"][d] = 0.0
    obs = gather_obs_ragged(torch.from_numpy(s["obs"]), BG)
    keys = [torch.empty(2, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(keys, torch.from_numpy(gkey.astype(np.int64)))
    flags = [None] * world
    dist.all_gather_object(flags, split_flags)
    if rank == 0:
        q.put((obs.numpy(), gkey, any_steps, [k.numpy() for k in keys], flags))
    dist.destroy_process_group()


def _gym_single(name, force=None):
    import orc
    import pob_np as P
    e = orc.OracleEnv(name)
    ks = P.split(P.prngkey(3), BG + 1)
    s, gkey = e.reset(ks[1:]), ks[0].copy()
    akey = P.prngkey(8)
    for t in range(TG):
        akey, k = P.split(akey)
        s = e.step(s, P.uniform(k, (BG, 8), -1, 1), flags=orc.F_EPISODE, episode_length=LG)
        if force is not None and t == force[0]:
            s["done"][force[1]] = 1.0
        e.gym_autoreset(s, gkey)
    return s["obs"], gkey


def test_sharded_gym_autoreset_equals_single_world2():
    ctx = mp.get_context("spawn")
    for name in ("ant_tag", "ant_heavenhell"):
        q = ctx.Queue()
        port = _free_port()
        procs = [ctx.Process(target=_gym_rank, args=(r, 2, port, name, q)) for r in range(2)]
        for p in procs:
            p.start()
        obs, gkey, any_steps, keys, _ = q.get(timeout=120)
        for p in procs:
            p.join(timeout=120)
            assert p.exitcode == 0
        assert any_steps >= 2  # the global key advanced on several steps
        want_obs, want_key = _gym_single(name)
        np.testing.assert_array_equal(obs, want_obs)
        np.testing.assert_array_equal(gkey, want_key)
        for k in keys:
            np.testing.assert_array_equal(k, want_key.astype(np.int64))


def test_sharded_gym_ranks_disagree_on_any_done():
    """Only rank 0 has a done env at step 1 (env 3 of 49 ends early, before the episode
    limit ends every env at step 3): rank 1's local any-done is 0 but the all-reduced flag
    is 1, so rank 1 must advance the gym key too and leave all its rows untouched.  A
    local-only any-done (or a dropped all-reduce) desynchronises rank 1's key, which this
    catches in every later reset and in the final keys of both ranks."""
    ctx = mp.get_context("spawn")
    name, force = "ant_tag", (1, 3)
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gym_rank, args=(r, 2, port, name, q, force)) for r in range(2)]
    for p in procs:
        p.start()
    obs, gkey, any_steps, keys, flags = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert (1, 0, 1) in flags[1]  # rank 1: nothing done locally, done globally at step 1
    want_obs, want_key = _gym_single(name, force)
    np.testing.assert_array_equal(obs, want_obs)
    for k in keys:
        np.testing.assert_array_equal(k, want_key.astype(np.int64))


# ---------------------------------------------------------------- overlapped obs gather
def _obs_at(t, lo, hi, D):
    """Synthetic obs of step t for global envs [lo, hi): a unique value per (t, env, col)."""
    i = torch.arange(lo, hi, dtype=torch.float32)[:, None]
    c = torch.arange(D, dtype=torch.float32)[None, :]
    return 1000.0 * t + 10.0 * i + c / D


def _gather_rank(rank, world, port, total, q):
    """The product's ObsGatherer (double-buffered obs, gather of step t overlapped with step
    t + 1) over gloo: after submitting step t, BOTH step t's and step t - 1's slots hold the
    full batches of their steps (slot rotation), and a slot is rewritten only by step t + 2."""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "po-brax_amd")]
    from po_brax_amd.sharding import ObsGatherer, shard_range
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    D = 5
    lo, hi = shard_range(total, world, rank)
    g = ObsGatherer(total, D, depth=2)
    ok, slots = True, []
    obs = torch.empty((hi - lo, D))
    for t in range(6):
        obs.copy_(_obs_at(t, lo, hi, D))  # the step kernel overwrites obs in place every step
        slots.append(g.submit(obs))
        ok &= torch.equal(g.result(slots[t]), _obs_at(t, 0, total, D))
        if t >= 1:  # the previous step's batch is still intact in the other slot
            ok &= torch.equal(g.result(slots[t - 1]), _obs_at(t - 1, 0, total, D))
    ok &= slots == [0, 1, 0, 1, 0, 1]
    res = [None] * world
    dist.all_gather_object(res, bool(ok))
    if rank == 0:
        q.put(res)
    dist.destroy_process_group()


def test_obs_gatherer_double_buffer_world2():
    ctx = mp.get_context("spawn")
    for total in (48, 49):  # equal and ragged shards
        q = ctx.Queue()
        port = _free_port()
        procs = [ctx.Process(target=_gather_rank, args=(r, 2, port, total, q)) for r in range(2)]
        for p in procs:
            p.start()
        res = q.get(timeout=120)
        for p in procs:
            p.join(timeout=120)
            assert p.exitcode == 0
        assert res == [True, True], total


def test_obs_gatherer_ragged_world4():
    """world 4 (gloo): ragged shards, including an empty one (total 3: 1 + 1 + 1 + 0), an
    uneven split (50 = 13 + 13 + 12 + 12) and an even one (48), through the same slot
    rotation: every step's gathered batch equals the global obs in env order."""
    ctx = mp.get_context("spawn")
    for total in (3, 50, 48):
        q = ctx.Queue()
        port = _free_port()
        procs = [ctx.Process(target=_gather_rank, args=(r, 4, port, total, q)) for r in range(4)]
        for p in procs:
            p.start()
        res = q.get(timeout=180)
        for p in procs:
            p.join(timeout=120)
            assert p.exitcode == 0
        assert res == [True] * 4, total
